# usage: bash tools/gpurun/r02_ab.sh TAG ROUNDS LIB... [-- bench args]  -- interleaved A/B bench lines of library
# variants (lodestar_amd/LIB), ROUNDS times each, no cpu baseline
TAG=$1; R=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
for i in $(seq 1 $R); do
  for L in "${LIBS[@]}"; do
    BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_${L%.so}_$i.json 2> gpurun_out/${TAG}_${L%.so}_$i.err || exit 1
  done
done
