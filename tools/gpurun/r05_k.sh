# usage: bash tools/gpurun/r05_k.sh TAG -- full GPU tests, curve (valid + 1% invalid), C1/C3/C5/C2 benches
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u tools/latency_curve.py --sizes 128,256,512,1024,2048,4096,8192,16384 --variants "r5:" \
  --load-steps 100 --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
timeout -k 10 300 python -u tools/latency_curve.py --sizes 512,1024,2048,4096,8192 --variants "r5:" --invalid 0.01 --jobs3 \
  --load-steps 100 --out gpurun_out/${TAG}_curve_inv.json > gpurun_out/${TAG}_curve_inv.log 2>&1
timeout -k 10 300 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline > gpurun_out/${TAG}_C5.json 2> gpurun_out/${TAG}_C5.err
timeout -k 10 300 python -u bench.py --config C1 --inflight 32 --steps 1000 --warmup 64 --no-cpu-baseline > gpurun_out/${TAG}_C1.json 2> gpurun_out/${TAG}_C1.err
timeout -k 10 300 python -u bench.py --config C3 --inflight 32 --steps 300 --warmup 32 --no-cpu-baseline > gpurun_out/${TAG}_C3.json 2> gpurun_out/${TAG}_C3.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_C2.json 2> gpurun_out/${TAG}_C2.err
