# usage: bash tools/gpurun/r05_j.sh TAG -- acc6 two-wave (default) vs one-wave variant: curve + C2
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "chunk" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u tools/latency_curve.py --sizes 512,1024,2048,4096,8192,16384 --pool 16384 \
  --variants "w2:" --load-steps 100 --out gpurun_out/${TAG}_curve_w2.json > gpurun_out/${TAG}_curve_w2.log 2>&1
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_w1.so timeout -k 10 300 python -u tools/latency_curve.py --sizes 512,1024,2048,4096,8192,16384 --pool 16384 \
  --variants "w1:" --load-steps 100 --out gpurun_out/${TAG}_curve_w1.json > gpurun_out/${TAG}_curve_w1.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C2.json 2> gpurun_out/${TAG}_C2.err
