# usage: bash tools/gpurun/r05_av.sh TAG -- idle_wait_us (burst lingering on an idle device) on the small-call
# configs at 32 calls in flight: C1 x {0, 300, 1000, 2000}, C3 / C5 x {0, 1000}, alternating
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--inflight 32 --no-cpu-baseline --no-parity"
for w in 0 300 1000 2000; do
  timeout -k 10 200 python -u bench.py --config C1 $B --steps 1000 --warmup 64 --idle-wait-us $w > gpurun_out/${TAG}_C1_w$w.json 2>/dev/null
done
for w in 0 1000; do
  timeout -k 10 200 python -u bench.py --config C3 $B --steps 300 --warmup 32 --idle-wait-us $w > gpurun_out/${TAG}_C3_w$w.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --config C5 $B --steps 400 --warmup 32 --idle-wait-us $w > gpurun_out/${TAG}_C5_w$w.json 2>/dev/null
done
