# usage: bash tools/gpurun/hwq.sh TAG "queue counts"  -- C2 bench with the box's HW-queue setting, then with
# GPU_MAX_HW_QUEUES set explicitly to each listed count
set -e
TAG=$1; LIST=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}" > gpurun_out/${TAG}_env.txt
timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_box.json 2> gpurun_out/${TAG}_box.err
for q in $LIST; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_q$q.json 2> gpurun_out/${TAG}_q$q.err
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 16 "$@" > gpurun_out/${TAG}_q${q}_if16.json 2> gpurun_out/${TAG}_q${q}_if16.err
done
