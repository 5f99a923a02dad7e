# usage: bash tools/gpurun/sweep.sh TAG "inflight list" [extra bench args]  -- throughput sweep over in-flight depth
set -e
TAG=$1; LIST=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for d in $LIST; do
  timeout -k 10 300 python bench.py --inflight $d --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench_if$d.json 2> gpurun_out/${TAG}_bench_if$d.err
done
