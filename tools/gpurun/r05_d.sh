# usage: bash tools/gpurun/r05_d.sh TAG -- C5 under load over slots x lane-form fallback checks
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for V in "--slots 3" "--slots 6" "--slots 3 --set fb_lane_min=256" "--slots 6 --set fb_lane_min=256" "--slots 8 --set fb_lane_min=256"; do
  i=$((i+1))
  echo "$V" > gpurun_out/${TAG}_C5_v$i.args
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 300 --warmup 32 --no-cpu-baseline --no-parity $V > gpurun_out/${TAG}_C5_v$i.json 2> gpurun_out/${TAG}_C5_v$i.err
done
