# usage: bash tools/gpurun/r05_c1.sh TAG -- C1 / C3 at 32 calls in flight vs the run-merging knobs (slots, merge wait,
# pipeline depth): bigger merged runs trade per-call latency for fill
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 200 python -u bench.py --steps 300 --warmup 32 --no-cpu-baseline --no-parity"
i=0
for C in C1 C3; do
  for A in "" "--slots 1" "--slots 2" "--merge-wait-us 6000" "--slots 1 --pipeline-depth 2" "--slots 2 --merge-wait-us 6000" "--slots 1 --merge-wait-us 6000"; do
    i=$((i+1))
    echo "$C $A" > gpurun_out/${TAG}_$i.args
    $B --config $C $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
