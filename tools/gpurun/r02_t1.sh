# usage: bash tools/gpurun/r02_t1.sh TAG PYTEST_ARGS... -- selected GPU tests (verbose, per-test timeout)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > gpurun_out/${TAG}_t1.log 2>&1
