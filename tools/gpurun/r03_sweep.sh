# usage: bash tools/gpurun/r03_sweep.sh TAG ROUNDS "ARGS1" "ARGS2" ...  -- interleaved bench lines of the default
# library under different bench/runtime arguments (no cpu baseline, no parity leg), ROUNDS times each
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  k=0
  for A in "$@"; do
    k=$((k+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_v${k}_$i.json 2> gpurun_out/${TAG}_v${k}_$i.err
  done
done
