# usage: bash tools/gpurun/r06_acc.sh TAG -- Miller accumulation forms of merged runs on C2 (100 steps, 2 rounds):
# default (one lane per chunk of 2), six lanes per pairing for every run (acc6_max 10^6), two lanes (miller_lanes 2)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "base:" "acc6:--set acc6_max=1000000" "lanes2:--set miller_lanes=2"; do
    name=${cfg%%:*}; opts=${cfg#*:}
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity $opts \
      > gpurun_out/${TAG}_${name}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
