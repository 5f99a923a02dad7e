# usage: bash tools/gpurun/r05_r.sh TAG -- aggregation lane-group parity; C4 / C3 benches (grouped vs one wave per set)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 250 --timeout-method thread -k "aggregate or c4 or c3" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C4.json 2> gpurun_out/${TAG}_C4.err
timeout -k 10 300 python -u bench.py --config C3 --inflight 32 --steps 300 --warmup 32 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C3.json 2> gpurun_out/${TAG}_C3.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_pk1.so timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C4_pk1.json 2> gpurun_out/${TAG}_C4_pk1.err
