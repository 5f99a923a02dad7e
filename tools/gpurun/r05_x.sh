# usage: bash tools/gpurun/r05_x.sh TAG -- lane-pair accumulation for runs beyond acc6_max (miller_pairs) and lane-pair
# lines (lines_lanes 2): C2 A/B, driver's 20-step command, two rounds
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity"
for r in a b; do
  $B --set miller_pairs=1 --lines-lanes 2 > gpurun_out/${TAG}_p1l2$r.json 2> gpurun_out/${TAG}_p1l2$r.err
  $B --set miller_pairs=0 > gpurun_out/${TAG}_p0l1$r.json 2> gpurun_out/${TAG}_p0l1$r.err
  $B --set miller_pairs=1 > gpurun_out/${TAG}_p1l1$r.json 2> gpurun_out/${TAG}_p1l1$r.err
done
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --set miller_pairs=1 --lines-lanes 2 > gpurun_out/${TAG}_p1l2c.json 2> gpurun_out/${TAG}_p1l2c.err
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --set miller_pairs=0 > gpurun_out/${TAG}_p0l1c.json 2> gpurun_out/${TAG}_p0l1c.err
