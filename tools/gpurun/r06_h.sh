# usage: bash tools/gpurun/r06_h.sh TAG -- the candidate library: the whole GPU suite and smoke, then the round-6
# evidence (r06_final.sh)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
bash tools/gpurun/r06_final.sh ${TAG}f
