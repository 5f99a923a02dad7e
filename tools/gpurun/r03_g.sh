# usage: bash tools/gpurun/r03_g.sh TAG -- GPU tests, two 100-step C2 lines, the driver's 20-step command, and the
# FETCH_SIZE / WRITE_SIZE PMC passes of the driver's command
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 100 --warmup 5 > gpurun_out/${TAG}_v1_$i.json 2> gpurun_out/${TAG}_v1_$i.err
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --steps 20 --warmup 5 > gpurun_out/${TAG}_v2_1.json 2> gpurun_out/${TAG}_v2_1.err
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
