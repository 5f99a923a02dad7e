# usage: bash tools/gpurun/r06_y.sh TAG -- C5 (2,000 steps) with the recalibrated adaptive groups vs fixed 32 / 64,
# 3 interleaved rounds; then the adaptive form with the parity leg, and the driver's C2 command (all valid: adapt
# keeps 1,024-set groups)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline \
    --no-parity --no-profile > gpurun_out/${TAG}_C5_adapt_r$rep.json 2>> gpurun_out/${TAG}.err
  for g in 32 64; do
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline \
      --no-parity --no-profile --set group_adapt=0 --group-sets $g > gpurun_out/${TAG}_C5_g${g}_r$rep.json \
      2>> gpurun_out/${TAG}.err
  done
done
timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 > gpurun_out/${TAG}_C5_final.json \
  2>> gpurun_out/${TAG}.err
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
  > gpurun_out/${TAG}_C2.json 2>> gpurun_out/${TAG}.err
