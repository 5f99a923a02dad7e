# usage: bash tools/gpurun/r06_x.sh TAG -- C5 (2,000 steps) by fixed batch-group size (group_adapt 0): 32 / 64 / 128 /
# 256 / 512 sets, 2 interleaved rounds
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for g in 32 64 128 256 512; do
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline \
      --no-parity --no-profile --set group_adapt=0 --group-sets $g > gpurun_out/${TAG}_C5_g${g}_r$rep.json \
      2>> gpurun_out/${TAG}.err
  done
done
