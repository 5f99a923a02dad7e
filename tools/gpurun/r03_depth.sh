# usage: bash tools/gpurun/r03_depth.sh TAG ROUNDS "ARGS"... -- the driver's command (C2, 20 steps, 5 warmup, no cpu
# baseline / parity leg) per extra-argument set, interleaved
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  k=0
  for A in "$@"; do
    k=$((k + 1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 $A > gpurun_out/${TAG}_v${k}_$i.json 2> gpurun_out/${TAG}_v${k}_$i.err
  done
done
