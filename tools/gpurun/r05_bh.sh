# usage: bash tools/gpurun/r05_bh.sh TAG -- final library: the driver's command with GPU_MAX_HW_QUEUES 4 (default)
# and 8 (three stream pairs), four rounds interleaved
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--gpus 1 --warmup 5 --steps 20 --no-cpu-baseline --no-parity"
for i in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py $B > gpurun_out/${TAG}_q4_$i.json 2>/dev/null
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py $B > gpurun_out/${TAG}_q8_$i.json 2>/dev/null
done
