# usage: bash tools/gpurun/r05_ao.sh TAG -- C5 fallback forms for small idle runs: cooperative direct checks (default)
# vs the loaded-run forms (six-lane final exponentiations; fb_force_busy) -- isolated p50 and 32-in-flight throughput
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for r in a b; do
  for A in "" "--set fb_force_busy=1" "--set fb_force_busy=1 --set fb_direct_min=1"; do
    i=$((i+1)); echo "C5 $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --config C5 --steps 300 --warmup 32 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
