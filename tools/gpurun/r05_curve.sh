# usage: bash tools/gpurun/r05_curve.sh TAG -- GPU tests (fallback + configs), then the isolated-latency / loaded
# throughput curve over the cooperative-form thresholds (tools/latency_curve.py), all-valid and C5-like 1% invalid
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
V='base:;c1k:coop_max=1024,coop_g2_max=1024;c2k:coop_max=2048,coop_g2_max=2048;c4k:coop_max=4096,coop_g2_max=4096;g8k:coop_max=2048,coop_g2_max=8192;x2k:coop_max=2048,coop_g2_max=2048,coop_excl_max=2048'
timeout -k 10 400 python -u tools/latency_curve.py --sizes 256,512,1024,2048,4096,8192,16384 --variants "$V" \
  --load-steps 200 --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
timeout -k 10 300 python -u tools/latency_curve.py --sizes 512,1024,2048,4096 --variants "base:;c2k:coop_max=2048,coop_g2_max=2048" \
  --invalid 0.01 --jobs3 --load-steps 100 --out gpurun_out/${TAG}_curve_inv.json > gpurun_out/${TAG}_curve_inv.log 2>&1
