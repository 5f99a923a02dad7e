# usage: bash tools/gpurun/r03_ab.sh TAG ROUNDS LIB... [-- bench args]  -- GPU tests on the default library, then
# interleaved A/B bench lines of library variants (lodestar_amd/LIB) at the box's default hardware queues, ROUNDS
# times each (no cpu baseline, no parity leg), then one WRITE_SIZE / FETCH_SIZE PMC pass of the default library
set -e
TAG=$1; R=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for i in $(seq 1 $R); do
  for L in "${LIBS[@]}"; do
    BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/${TAG}_${L%.so}_$i.json 2> gpurun_out/${TAG}_${L%.so}_$i.err
  done
done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
