# usage: bash tools/gpurun/r02_ilp_q16.sh TAG  -- the ILP / code-size microbenchmark, then ONE bench run with
# GPU_MAX_HW_QUEUES=16 (the round-1 abort configuration), last because it may abort
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 180 tools/microbench/ilp_rate > gpurun_out/${TAG}_ilp.json 2> gpurun_out/${TAG}_ilp.err
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --slots 16 --inflight 32 > gpurun_out/${TAG}_q16.json 2> gpurun_out/${TAG}_q16.err
