# usage: bash tools/gpurun/r06_z.sh TAG -- merged-run cap on the driver's C2 command: merge_sets 98,304 / 131,072 /
# 163,840 (6 / 8 / 10 calls), 3 interleaved rounds at 20 steps, 1 at 100
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  for m in 131072 98304 163840; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --merge-sets $m > gpurun_out/${TAG}_m${m}_20_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
for m in 131072 98304 163840; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
    --merge-sets $m > gpurun_out/${TAG}_m${m}_100_r1.json 2>> gpurun_out/${TAG}.err
done
