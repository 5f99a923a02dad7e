# usage: bash tools/gpurun/r05_bg.sh TAG -- options test on the final tree, then the driver's command ten times
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_options.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
bash tools/gpurun/r05_az.sh ${TAG}
