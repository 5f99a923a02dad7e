# usage: bash tools/gpurun/r02_slots.sh TAG  -- bench lines (no cpu baseline) over runtime slots / merged runs and
# miller_k, under the box's own environment (bench.py raises GPU_MAX_HW_QUEUES to 8)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err; }
run base
run s2 --slots 2
run s3 --slots 3
run s4 --slots 4
run s2m128 --slots 2 --merge-sets 131072 --inflight 16
run s4i24 --slots 4 --inflight 24
run k3 --miller-k 3
run k4 --miller-k 4
run k1 --miller-k 1
