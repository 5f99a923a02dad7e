# usage: bash tools/gpurun/r05_bf.sh TAG -- spec_large: parity tests (the new spec test + options), then the driver's
# command five rounds interleaved with and without it, 100 steps each, and C4 / C5 single runs
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py -m gpu -x -v --timeout 240 --timeout-method thread -k "speculative or option or full_size" > gpurun_out/${TAG}_tests.log 2>&1
B="--gpus 1 --warmup 5 --no-cpu-baseline --no-parity"
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py $B --steps 20 > gpurun_out/${TAG}_base_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py $B --steps 20 --set spec_large=1 > gpurun_out/${TAG}_sl_$i.json 2>/dev/null
done
timeout -k 10 200 python -u bench.py $B --steps 100 > gpurun_out/${TAG}_base_100.json 2>/dev/null
timeout -k 10 200 python -u bench.py $B --steps 100 --set spec_large=1 > gpurun_out/${TAG}_sl_100.json 2>/dev/null
timeout -k 10 300 python -u bench.py --gpus 1 --warmup 5 --steps 20 --no-cpu-baseline --set spec_large=1 > gpurun_out/${TAG}_sl_parity.json 2>/dev/null
