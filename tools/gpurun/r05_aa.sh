# usage: bash tools/gpurun/r05_aa.sh TAG -- r_i pk_i (k_pk_finish) and hash_to_field (k_hash_prep) at two waves per
# SIMD: parity (pipeline + C3/C4 configs) and C2 / C4 A/B against k_pk_finish at one wave (libblsgpu_pk1.so)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_golden.py -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity"
for r in a b; do
  $B > gpurun_out/${TAG}_n$r.json 2> gpurun_out/${TAG}_n$r.err
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_pk1.so $B > gpurun_out/${TAG}_o$r.json 2> gpurun_out/${TAG}_o$r.err
done
B="timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity"
$B > gpurun_out/${TAG}_nc.json 2> gpurun_out/${TAG}_nc.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_pk1.so $B > gpurun_out/${TAG}_oc.json 2> gpurun_out/${TAG}_oc.err
B="timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity"
$B > gpurun_out/${TAG}_n4.json 2> gpurun_out/${TAG}_n4.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_pk1.so $B > gpurun_out/${TAG}_o4.json 2> gpurun_out/${TAG}_o4.err
