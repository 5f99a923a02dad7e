# usage: bash tools/gpurun/r03_trace2.sh TAG LIB... -- rocprofv3 kernel traces of the bench (100 steps) per library
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${L%.so} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${L%.so}.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${L%.so}.log
done
