# usage: bash tools/gpurun/r02_sweep2.sh TAG "ARGS1" "ARGS2" ...  -- one bench line (no cpu baseline) per argument
# set, each under its own time limit; stops at the first failure
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
i=0
for a in "$@"; do
  echo "== $a" >> gpurun_out/${TAG}_sweep.log
  timeout -k 10 120 python bench.py --no-cpu-baseline $a >> gpurun_out/${TAG}_sweep.log 2> gpurun_out/${TAG}_sweep_$i.err
  i=$((i+1))
done
