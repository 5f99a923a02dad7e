# usage: bash tools/gpurun/r02_vbench.sh TAG LIB...  -- one bench line per library variant (no cpu baseline)
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
for L in "$@"; do
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_$L.json 2> gpurun_out/${TAG}_$L.err || true
done
