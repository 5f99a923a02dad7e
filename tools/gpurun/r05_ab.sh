# usage: bash tools/gpurun/r05_ab.sh TAG -- hash_to_field at two waves (k_hash_prep) and the MSM window sums / slice
# tree on lane pairs: parity (MSM forms, pipeline) + C2 A/B, three interleaved rounds of 100 steps
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_midsize.py tests/test_gpu_pipeline.py -x -v --timeout 250 --timeout-method thread -k "msm or slice or 8192 or 4096 or exceptional or verify or hash" > gpurun_out/${TAG}_tests.log 2>&1
B="timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity"
for r in a b c; do
  $B > gpurun_out/${TAG}_n$r.json 2> gpurun_out/${TAG}_n$r.err
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_h1.so $B > gpurun_out/${TAG}_h$r.json 2> gpurun_out/${TAG}_h$r.err
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_w0.so $B > gpurun_out/${TAG}_w$r.json 2> gpurun_out/${TAG}_w$r.err
done
