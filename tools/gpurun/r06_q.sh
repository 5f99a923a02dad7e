# usage: bash tools/gpurun/r06_q.sh TAG -- urgent streams created on the lane's first call (no idle hardware queues
# otherwise): the urgent / option / fault tests; the driver's C2 command against the eager build
# (variants/libv_ueager.so, r06_f.sh); the 8-context host-capacity mode both ways
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_urgent.py tests/test_gpu_options.py tests/test_gpu_faults.py \
  tests/test_gpu_api.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
bash tools/gpurun/r06_f.sh ${TAG} base ueager
for v in base ueager; do
  L=lodestar_amd/libblsgpu.so; [ "$v" = base ] || L=lodestar_amd/variants/libv_$v.so
  BLSGPU_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --gpus 8 --devices-same 0 --inflight 8 --steps 20 \
    --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_host8_${v}.json 2>> gpurun_out/${TAG}.err
done
