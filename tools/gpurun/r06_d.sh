# usage: bash tools/gpurun/r06_d.sh TAG -- urgent lane on dedicated CU-masked queues: the urgent tests; urgent latency
# under a 200-step C2 flood (default lane, plain high-priority streams, the isolated 8-CU partition); the driver's
# command x3; a kernel trace of isolated urgent calls; the whole GPU suite; the hash-TU scheduler variants (r06_f.sh)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_urgent.py -v -s --timeout 240 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for cfg in "0 1" "0 2" "8 1"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
    --urgent-every-ms 10 --set urgent_cus=$1 --set urgent_isolate=$2 > gpurun_out/${TAG}_lat_u$1_i$2.json \
    2>> gpurun_out/${TAG}_lat.err
done
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    > gpurun_out/${TAG}_c2_r$rep.json 2>> gpurun_out/${TAG}_c2.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_utrace -o run \
  -- python3 $GRAFT_REPO_ROOT/tools/urgent_latency.py --reps 10 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_utrace.log 2>&1
cd $GRAFT_REPO_ROOT
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/gpurun/r06_f.sh ${TAG}v base noilp mix
