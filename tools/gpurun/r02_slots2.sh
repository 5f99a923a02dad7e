# usage: bash tools/gpurun/r02_slots2.sh TAG  -- the ILP microbenchmark, then bench lines (no cpu baseline) over
# runtime slots x calls in flight x merged-run size
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench/ilp_rate > gpurun_out/${TAG}_ilp.json 2> gpurun_out/${TAG}_ilp.err
run() { local name=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err; }
run s4i24 --slots 4 --inflight 24
run s4i32 --slots 4 --inflight 32
run s4i48 --slots 4 --inflight 48
run s4i32m128 --slots 4 --inflight 32 --merge-sets 131072
run s3i24 --slots 3 --inflight 24
run s6i36 --slots 6 --inflight 36
run s2i24m128 --slots 2 --inflight 24 --merge-sets 131072
run s4i32k1 --slots 4 --inflight 32 --miller-k 1
run s4i32k3 --slots 4 --inflight 32 --miller-k 3
