# usage: bash tools/gpurun/r02_sweep.sh TAG  -- GPU tests, then bench lines over miller_k (no cpu baseline)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for K in 1 2 4 8; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --miller-k $K > gpurun_out/${TAG}_k$K.json 2> gpurun_out/${TAG}_k$K.err
done
