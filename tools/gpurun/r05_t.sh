# usage: bash tools/gpurun/r05_t.sh TAG -- lane-pair cofactor clearing: parity (8k mid-size, C2 parity leg) and C2 A/B
# against the one-lane build (libblsgpu_h1.so), the driver's 20-step command and 100 steps
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_midsize.py -x -v --timeout 250 --timeout-method thread -k "8192 or all_valid" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_new20.json 2> gpurun_out/${TAG}_new20.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_h1.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_old20.json 2> gpurun_out/${TAG}_old20.err
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_new100.json 2> gpurun_out/${TAG}_new100.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_h1.so timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_old100.json 2> gpurun_out/${TAG}_old100.err
