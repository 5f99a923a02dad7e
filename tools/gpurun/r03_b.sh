# usage: bash tools/gpurun/r03_b.sh TAG -- GPU tests, the driver's bench command, then a hardware-queue / slots sweep
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
for S in 1 2 4; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --slots $S --no-cpu-baseline --no-parity > gpurun_out/${TAG}_q4s$S.json 2>> gpurun_out/${TAG}_sweep.err
done
for S in 2 4; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --slots $S --no-cpu-baseline --no-parity > gpurun_out/${TAG}_q8s$S.json 2>> gpurun_out/${TAG}_sweep.err
done
for S in 1 2 4; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 5 --slots $S --no-cpu-baseline --no-parity > gpurun_out/${TAG}_q4s${S}_200.json 2>> gpurun_out/${TAG}_sweep.err
done
