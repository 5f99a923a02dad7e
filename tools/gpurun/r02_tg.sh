# usage: bash tools/gpurun/r02_tg.sh TAG  -- GPU tests + smoke, then bench lines over group sizes (K=2)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
for G in 256 512; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --group-sets $G > gpurun_out/${TAG}_g$G.json 2> gpurun_out/${TAG}_g$G.err
done
