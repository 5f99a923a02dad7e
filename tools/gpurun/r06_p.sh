# usage: bash tools/gpurun/r06_p.sh TAG -- LDS-staged line prefetch in the Miller accumulation: the parity suites that
# run every accumulation form (chunk forms, mid-size forms, pipeline stages), then the driver's C2 command against the
# library built without it (variants/libv_nopre.so), 3 rounds at 20 steps and 2 at 100 (r06_f.sh); C4 both ways
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_midsize.py tests/test_gpu_pipeline.py \
  tests/test_gpu_configs.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
bash tools/gpurun/r06_f.sh ${TAG} base nopre
for rep in 1 2; do
  for v in base nopre; do
    L=lodestar_amd/libblsgpu.so; [ "$v" = base ] || L=lodestar_amd/variants/libv_$v.so
    BLSGPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 \
      --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C4_${v}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
