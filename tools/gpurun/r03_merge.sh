# usage: bash tools/gpurun/r03_merge.sh TAG ROUNDS MERGE... -- GPU tests, then the driver's command (C2, 20 steps,
# 5 warmup, no cpu baseline / parity leg) per merge_sets value, interleaved
set -e
TAG=$1; R=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for i in $(seq 1 $R); do
  for M in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 --merge-sets $M > gpurun_out/${TAG}_m${M}_$i.json 2> gpurun_out/${TAG}_m${M}_$i.err
  done
done
