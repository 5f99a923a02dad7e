# usage: bash tools/gpurun/r05_ac.sh TAG -- Miller chunk size on merged runs (shared squarings: 19 Fp2 products per
# pairing-step at k = 2 against 25 at k = 1) with the one-lane / two-lane / lane-pair accumulations: C2, 100 steps
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity"
for r in a b; do
  $B > gpurun_out/${TAG}_d$r.json 2> gpurun_out/${TAG}_d$r.err
  $B --miller-k 2 > gpurun_out/${TAG}_k2$r.json 2> gpurun_out/${TAG}_k2$r.err
  $B --miller-k 2 --set miller_pairs=1 > gpurun_out/${TAG}_k2p$r.json 2> gpurun_out/${TAG}_k2p$r.err
  $B --miller-k 4 --set miller_pairs=1 > gpurun_out/${TAG}_k4p$r.json 2> gpurun_out/${TAG}_k4p$r.err
done
