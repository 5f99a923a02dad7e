# usage: bash tools/gpurun/r02_bpmc.sh TAG  -- GPU tests, the default bench line (with cpu baseline), rocprof
# kernel stats of the same command, then the two PMC traffic passes (tools/gpurun/r02_pmc.sh)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
bash $GRAFT_REPO_ROOT/tools/gpurun/r02_pmc.sh $TAG
