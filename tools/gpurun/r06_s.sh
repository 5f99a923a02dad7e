# usage: bash tools/gpurun/r06_s.sh TAG -- C5 (2,000 steps) by batch-group size: adaptive (default) vs fixed groups of
# >= 1 / 4 / 16 / 64 sets (group_adapt 0), 2 interleaved rounds, with the parity leg on the first round
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  P="--no-parity"; [ $rep = 1 ] && P=""
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline $P \
    --no-profile > gpurun_out/${TAG}_C5_adapt_r$rep.json 2>> gpurun_out/${TAG}.err
  for g in 1 4 16 64; do
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline $P \
      --no-profile --set group_adapt=0 --group-sets $g > gpurun_out/${TAG}_C5_g${g}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
