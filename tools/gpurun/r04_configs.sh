# usage: bash tools/gpurun/r04_configs.sh TAG [configs...]  -- one bench line per BASELINE config at this build, each with
# its parity leg and cpu_baseline (C2 = the driver's command; C1 with 32 calls in flight; C4 = all 32,768 sets on one
# device).  Progress lines go to gpurun_out/${TAG}_progress.txt.
set -e
TAG=$1; shift
CFGS=${@:-"C2 C1 C3 C4 C5"}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for C in $CFGS; do
  echo "$(date +%T) start $C" >> gpurun_out/${TAG}_progress.txt
  case $C in
    C2) ARGS="--gpus 1 --steps 20 --warmup 5" ;;
    C1) ARGS="--config C1 --inflight 32 --steps 2000 --warmup 64" ;;
    C3) ARGS="--config C3 --inflight 32 --steps 400 --warmup 32" ;;
    C4) ARGS="--config C4 --gpus 1 --inflight 8 --steps 40 --warmup 8" ;;
    C5) ARGS="--config C5 --inflight 32 --steps 800 --warmup 32" ;;
  esac
  timeout -k 10 420 python -u bench.py $ARGS > gpurun_out/${TAG}_bench_$C.json 2> gpurun_out/${TAG}_bench_$C.err
  echo "$(date +%T) done $C" >> gpurun_out/${TAG}_progress.txt
done
