# usage: bash tools/gpurun/r05_ap.sh TAG -- three stream pairs (GPU_MAX_HW_QUEUES=8: a pair per slot) vs two (the
# default 4 queues): parity under 8 queues, C2 at 20 (x3) / 100 steps, C1, C5
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_midsize.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests8.log 2>&1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_par8.json 2> gpurun_out/${TAG}_par8.err
i=0
for r in a b c; do
  for Q in 4 8; do
    i=$((i+1)); echo "20 q$Q" > gpurun_out/${TAG}_$i.args
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
for Q in 4 8; do
  i=$((i+1)); echo "100 q$Q" > gpurun_out/${TAG}_$i.args
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  for C in C1 C5; do
    i=$((i+1)); echo "$C q$Q" > gpurun_out/${TAG}_$i.args
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u bench.py --config $C --steps 300 --warmup 32 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
