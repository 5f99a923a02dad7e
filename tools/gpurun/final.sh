# usage: bash tools/gpurun/final.sh TAG  -- GPU tests, smoke, C2 bench at the defaults and over group sizes,
# then the rocprof kernel-stats pass of the default bench
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
for G in 512 1024; do
  timeout -k 10 200 python bench.py --group-sets $G --no-cpu-baseline > gpurun_out/${TAG}_bench_g$G.json 2> gpurun_out/${TAG}_bench_g$G.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
