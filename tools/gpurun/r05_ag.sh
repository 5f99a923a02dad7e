# usage: bash tools/gpurun/r05_ag.sh TAG -- merged runs larger than 131,072 sets (C2, 20 and 100 steps)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for S in 20 100; do
  for A in "" "--merge-sets 196608" "--merge-sets 262144" "--merge-sets 196608 --pipeline-depth 2"; do
    i=$((i+1))
    echo "$S $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --steps $S --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
