# usage: bash tools/gpurun/r05_af.sh TAG -- merged-run size vs runs in flight for C2 (20 and 100 steps)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for S in 20 100; do
  for A in "" "--merge-sets 65536" "--merge-sets 65536 --pipeline-depth 4 --slots 4" "--merge-sets 49152 --pipeline-depth 5 --slots 5" "--merge-sets 98304 --pipeline-depth 4 --slots 4"; do
    i=$((i+1))
    echo "$S $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --steps $S --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
