# usage: bash tools/gpurun/r06_c1.sh TAG -- C1 (128-set calls, 32 in flight, 5,000 steps) by run concurrency: slots /
# pipeline depth / merge wait (us): 3/3/2000 (default), 3/3/500, 4/4/500, 6/6/500, 6/6/0, 4/4/2000; 2 rounds; then C3
# with the best two
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "3 3 2000" "3 3 500" "4 4 500" "6 6 500" "6 6 0" "4 4 2000"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --config C1 --inflight 32 --steps 5000 --warmup 64 --no-cpu-baseline \
      --no-parity --no-profile --slots $1 --pipeline-depth $2 --merge-wait-us $3 \
      > gpurun_out/${TAG}_C1_s$1_d$2_w$3_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
