# usage: bash tools/gpurun/pmc.sh TAG [bench args...]  -- GPU tests, then HBM-traffic PMC passes (one counter
# group per pass, kernel-trace only, no sys/runtime trace) over a short serial bench run.
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-profile "$@" > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
