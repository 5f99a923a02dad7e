# usage: bash tools/gpurun/r03_e.sh TAG -- GPU tests, smoke, the driver's bench command, one 16-queue run,
# a rocprofv3 kernel-trace summary of exactly the driver's command, and FETCH_SIZE / WRITE_SIZE PMC passes
# of the same command (one counter per pass, kernel trace only).
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_q16.json 2> gpurun_out/${TAG}_q16.err
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_200.json 2> gpurun_out/${TAG}_200.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
