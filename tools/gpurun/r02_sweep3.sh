# usage: bash tools/gpurun/r02_sweep3.sh TAG "LIB|ARGS" ...  -- one bench line (no cpu baseline) per entry, with
# BLSGPU_LIB=lodestar_amd/LIB (a tuning variant; "-" = the product library); stops at the first failure
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
i=0
for e in "$@"; do
  lib=${e%%|*}; a=${e#*|}
  echo "== $lib | $a" >> gpurun_out/${TAG}_sweep.log
  if [ "$lib" = "-" ]; then unset BLSGPU_LIB; else export BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$lib; fi
  timeout -k 10 150 python bench.py --no-cpu-baseline $a >> gpurun_out/${TAG}_sweep.log 2> gpurun_out/${TAG}_sweep_$i.err
  i=$((i+1))
done
