# usage: bash tools/gpurun/r05_u.sh TAG -- lane-pair subgroup check + two-wave maps: parity (mid-size, pipeline,
# parity suites) and C2 A/B: new build, hash pairs only (libblsgpu_hp.so), one-lane build (libblsgpu_h1.so)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_midsize.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
$B > gpurun_out/${TAG}_new20a.json 2> gpurun_out/${TAG}_new20a.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_hp.so $B --no-parity > gpurun_out/${TAG}_hp20a.json 2> gpurun_out/${TAG}_hp20a.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_h1.so $B --no-parity > gpurun_out/${TAG}_h120a.json 2> gpurun_out/${TAG}_h120a.err
$B --no-parity > gpurun_out/${TAG}_new20b.json 2> gpurun_out/${TAG}_new20b.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_hp.so $B --no-parity > gpurun_out/${TAG}_hp20b.json 2> gpurun_out/${TAG}_hp20b.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_h1.so $B --no-parity > gpurun_out/${TAG}_h120b.json 2> gpurun_out/${TAG}_h120b.err
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_new100.json 2> gpurun_out/${TAG}_new100.err
