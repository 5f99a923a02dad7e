# usage: bash tools/gpurun/cfg.sh TAG  -- GPU tests, then short bench lines for C3/C4/C5 (parity-checked)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for C in C5 C3 C4; do
  timeout -k 10 300 python bench.py --config $C --steps 6 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench_$C.json 2> gpurun_out/${TAG}_bench_$C.err
done
