# usage: bash tools/gpurun/r05_l.sh TAG -- fallback parity tests, invalid curve, C5 bench
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_midsize.py tests/test_gpu_configs.py tests/test_gpu_faults.py -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u tools/latency_curve.py --sizes 512,1024,2048,4096,8192 --variants "r5:" --invalid 0.01 --jobs3 \
  --load-steps 100 --out gpurun_out/${TAG}_curve_inv.json > gpurun_out/${TAG}_curve_inv.log 2>&1
timeout -k 10 300 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline > gpurun_out/${TAG}_C5.json 2> gpurun_out/${TAG}_C5.err
