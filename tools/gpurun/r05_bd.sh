# usage: bash tools/gpurun/r05_bd.sh TAG -- GPU_MAX_HW_QUEUES=8 vs 4 at 100 steps (two rounds) and on C1 / C5 / C4
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--gpus 1 --warmup 5 --steps 100 --no-cpu-baseline --no-parity"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $B > gpurun_out/${TAG}_q4_100_$i.json 2>/dev/null
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py $B --set alone_msm=1 > gpurun_out/${TAG}_q8_100_$i.json 2>/dev/null
done
S="--inflight 32 --no-cpu-baseline --no-parity"
timeout -k 10 200 python -u bench.py --config C1 $S --steps 1000 --warmup 64 > gpurun_out/${TAG}_q4_C1.json 2>/dev/null
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --config C1 $S --steps 1000 --warmup 64 --set alone_msm=1 > gpurun_out/${TAG}_q8_C1.json 2>/dev/null
timeout -k 10 200 python -u bench.py --config C5 $S --steps 400 --warmup 32 > gpurun_out/${TAG}_q4_C5.json 2>/dev/null
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --config C5 $S --steps 400 --warmup 32 --set alone_msm=1 > gpurun_out/${TAG}_q8_C5.json 2>/dev/null
timeout -k 10 200 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_q4_C4.json 2>/dev/null
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity --set alone_msm=1 > gpurun_out/${TAG}_q8_C4.json 2>/dev/null
