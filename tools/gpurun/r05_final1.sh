# usage: bash tools/gpurun/r05_final1.sh TAG -- round-5 final build: full GPU suite + smoke, then the driver command's
# evidence (kernel trace + stats, FETCH_SIZE / WRITE_SIZE PMC passes, SQ counter pass; each its own run)
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
bash tools/gpurun/r05_evidence.sh ${TAG}e
