# usage: bash tools/gpurun/r06_c.sh TAG -- urgent lane: the flood test; throughput A/B of the lane's stream
# configurations (interleaved, the driver's 20 steps); urgent latency under a 200-step flood
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_urgent.py -v -s --timeout 240 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for rep in 1 2 3; do
  for cfg in "0 1" "8 0" "8 3" "8 1"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --set urgent_cus=$1 --set urgent_isolate=$2 > gpurun_out/${TAG}_ab_u$1_i$2_r$rep.json 2>> gpurun_out/${TAG}_ab.err
  done
done
for cfg in "0 1" "8 0" "8 1"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
    --urgent-every-ms 10 --set urgent_cus=$1 --set urgent_isolate=$2 > gpurun_out/${TAG}_lat_u$1_i$2.json \
    2>> gpurun_out/${TAG}_lat.err
done
