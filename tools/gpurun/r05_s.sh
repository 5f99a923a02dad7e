# usage: bash tools/gpurun/r05_s.sh TAG -- full GPU suite and smoke on the current build
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
