# usage: bash tools/gpurun/r02_head.sh TAG  -- GPU tests + smoke, the default bench line under the box's own
# GPU_MAX_HW_QUEUES (what the driver sees) and with 8, then the rocprof kernel-stats pass of the default bench
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" > gpurun_out/${TAG}_env.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench_q8.json 2> gpurun_out/${TAG}_bench_q8.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
