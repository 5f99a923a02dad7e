# usage: bash tools/gpurun/r06_a.sh TAG -- round 6, first urgent-lane pass: the urgent-lane, option and large-failing-job
# tests, then the driver's C2 command with the urgent latency probe under several lane configurations
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rc=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_urgent.py tests/test_gpu_options.py tests/test_gpu_midsize.py \
  -k "urgent or option or large_failing" -v -s --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc   # test failures (1) are read afterwards; a crash or time limit ends the call
for cfg in "0 1" "8 1" "8 2" "16 1" "8 0"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --urgent-every-ms 20 \
    --set urgent_cus=$1 --set urgent_isolate=$2 > gpurun_out/${TAG}_c2_u$1_i$2.json 2> gpurun_out/${TAG}_c2_u$1_i$2.err
done
