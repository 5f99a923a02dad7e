# usage: bash tools/gpurun/r02_bisect.sh TAG LIB...  -- golden + pipeline GPU tests against library variants
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
for L in "$@"; do
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_pipeline.py -m gpu -q --tb=line --timeout 100 --timeout-method thread -k "not js" > gpurun_out/${TAG}_$L.log 2>&1 || true
done
