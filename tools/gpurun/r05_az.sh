# usage: bash tools/gpurun/r05_az.sh TAG -- the driver's command ten times on one box (spread of the 20-step C2 metric)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2>/dev/null
done
