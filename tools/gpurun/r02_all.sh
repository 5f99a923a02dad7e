# usage: bash tools/gpurun/r02_all.sh TAG  -- every GPU test (no -x), short tracebacks
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python -u -m pytest tests -m gpu -q --tb=line --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || true
