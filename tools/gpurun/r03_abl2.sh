# usage: bash tools/gpurun/r03_abl2.sh TAG ROUNDS LIB... -- GPU tests (default library), serial C1 / C3 kernel traces
# (default library), then interleaved 100-step C2 lines of the libraries
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
bash tools/gpurun/r03_lat.sh $TAG C1 C3
cd $GRAFT_REPO_ROOT
for i in $(seq 1 $R); do
  for L in "$@"; do
    BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 5 > gpurun_out/${TAG}_${L%.so}_$i.json 2> gpurun_out/${TAG}_${L%.so}_$i.err
  done
done
