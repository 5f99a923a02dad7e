# usage: bash tools/gpurun/sweep.sh TAG "inflight list" [extra bench args]  -- throughput sweep over in-flight depth
set -e
TAG=$1; LIST=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for d in $LIST; do
  timeout -k 10 300 python bench.py --inflight $d --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench_if$d.json 2> gpurun_out/${TAG}_bench_if$d.err
done
if [ -n "$PROF_IF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --inflight $PROF_IF --steps 8 --warmup 1 --no-cpu-baseline --no-profile "$@" > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
fi
