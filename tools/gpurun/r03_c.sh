# usage: bash tools/gpurun/r03_c.sh TAG -- GPU tests, the driver's bench command, a slots sweep at the box's default
# hardware queues (+ one 8-queue line), and a rocprofv3 kernel trace of the driver's command
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
for S in 1 2 4 6; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --slots $S --no-cpu-baseline --no-parity > gpurun_out/${TAG}_q4s$S.json 2>> gpurun_out/${TAG}_sweep.err
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_q8.json 2>> gpurun_out/${TAG}_sweep.err
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_200.json 2>> gpurun_out/${TAG}_sweep.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log
