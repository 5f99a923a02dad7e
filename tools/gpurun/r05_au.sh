# usage: bash tools/gpurun/r05_au.sh TAG -- mid-size parity (512 / 513 edge) and a C5 A/B of the cooperative edge
# (default 512 vs coop_max 384), alternating, two runs each
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_midsize.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_c512_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline --no-parity --set coop_max=384 > gpurun_out/${TAG}_c384_$i.json 2>/dev/null
done
