# usage: bash tools/gpurun/r05_ba.sh TAG -- alone_msm A/B: the driver's command five rounds interleaved, 100 steps
# each, one run with the parity leg on, and isolated p50 (bench's p50_batch_latency_ms)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--gpus 1 --warmup 5 --no-cpu-baseline --no-parity"
timeout -k 10 300 python -u bench.py --gpus 1 --warmup 5 --steps 20 --no-cpu-baseline --set alone_msm=1 > gpurun_out/${TAG}_parity.json 2>/dev/null
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py $B --steps 20 > gpurun_out/${TAG}_base_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py $B --steps 20 --set alone_msm=1 > gpurun_out/${TAG}_am_$i.json 2>/dev/null
done
timeout -k 10 200 python -u bench.py $B --steps 100 > gpurun_out/${TAG}_base_100.json 2>/dev/null
timeout -k 10 200 python -u bench.py $B --steps 100 --set alone_msm=1 > gpurun_out/${TAG}_am_100.json 2>/dev/null
