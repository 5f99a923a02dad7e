# usage: bash tools/gpurun/r05_ae.sh TAG -- run formation for a burst (the driver's 20 calls arrive at once): idle
# wait (merge the burst on an idle device), balanced cuts, at 20 and 100 steps
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for S in 20 100; do
  for A in "" "--idle-wait-us 400" "--idle-wait-us 400 --merge-balance 1" "--merge-balance 1" "--idle-wait-us 2000 --merge-balance 1"; do
    i=$((i+1))
    echo "$S $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --steps $S --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
