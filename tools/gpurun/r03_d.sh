# usage: bash tools/gpurun/r03_d.sh TAG -- GPU tests, the driver's bench command, run-formation variants, a trace
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity"
timeout -k 10 200 $B --pipeline-depth 3 > gpurun_out/${TAG}_d3.json 2>> gpurun_out/${TAG}_sweep.err
timeout -k 10 200 $B --merge-wait-us 0 > gpurun_out/${TAG}_w0.json 2>> gpurun_out/${TAG}_sweep.err
timeout -k 10 200 $B --merge-wait-us 5000 > gpurun_out/${TAG}_w5.json 2>> gpurun_out/${TAG}_sweep.err
timeout -k 10 200 $B --slots 2 > gpurun_out/${TAG}_s2.json 2>> gpurun_out/${TAG}_sweep.err
timeout -k 10 200 $B --merge-sets 65536 > gpurun_out/${TAG}_m64.json 2>> gpurun_out/${TAG}_sweep.err
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_200.json 2>> gpurun_out/${TAG}_sweep.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log
