# usage: bash tools/gpurun/r03_ab2.sh TAG ROUNDS LIB... -- GPU tests (default library), interleaved C2 A/B lines
# (100 steps) of the libraries, then C1 and C3 lines (isolated-call latency) of each
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for i in $(seq 1 $R); do
  for L in "$@"; do
    BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 5 > gpurun_out/${TAG}_${L%.so}_$i.json 2> gpurun_out/${TAG}_${L%.so}_$i.err
  done
done
for L in "$@"; do
  for C in C1 C3; do
    BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --config $C --steps 200 --warmup 2 > gpurun_out/${TAG}_${C}_${L%.so}.json 2> gpurun_out/${TAG}_${C}_${L%.so}.err
  done
done
