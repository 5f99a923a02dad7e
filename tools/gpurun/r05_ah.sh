# usage: bash tools/gpurun/r05_ah.sh TAG -- early in-flight release (a run leaves the pipeline count when its message
# branch is done) with more slots: C2 at 20 and 100 steps; C1 at 300
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for S in 20 100; do
  for A in "" "--set early_release=1 --slots 4" "--slots 4" "--set early_release=1" "--set early_release=1 --slots 5 --pipeline-depth 4"; do
    i=$((i+1))
    echo "$S $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --steps $S --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
for A in "" "--set early_release=1 --slots 4"; do
  i=$((i+1))
  echo "C1 $A" > gpurun_out/${TAG}_$i.args
  timeout -k 10 300 python -u bench.py --config C1 --steps 300 --warmup 32 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
done
