# usage: bash tools/gpurun/r06_m.sh TAG -- spec_gsm (a speculative run's MillerLoop(-g1, S) behind its MSM on the other
# pair's message stream): the parity / option / urgent tests; the driver's C2 command with spec_gsm 1 / 0 and
# spec_gsm 1 + copy_stream 1 (4 interleaved rounds); C4 and C1 at 32 in flight (2 rounds); the isolated latency curve
# of both; a kernel trace of the driver's command with spec_gsm 1
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rc=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_options.py tests/test_gpu_urgent.py -v -s \
  --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for rep in 1 2 3 4; do
  for cfg in "1 0" "0 0" "1 1"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --set spec_gsm=$1 --set copy_stream=$2 > gpurun_out/${TAG}_C2_g$1_c$2_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
for rep in 1 2; do
  for g in 1 0; do
    timeout -k 10 200 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity \
      --no-profile --set spec_gsm=$g > gpurun_out/${TAG}_C4_g${g}_r$rep.json 2>> gpurun_out/${TAG}.err
    timeout -k 10 200 python -u bench.py --config C1 --inflight 32 --steps 1000 --warmup 64 --no-cpu-baseline \
      --no-parity --no-profile --set spec_gsm=$g > gpurun_out/${TAG}_C1_g${g}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
timeout -k 10 300 python -u tools/latency_curve.py --sizes 1,128,1024,4096,16384 \
  --variants "gsm1:spec_gsm=1;gsm0:spec_gsm=0" --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 \
  $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $R/gpurun_out/${TAG}_trace.json \
  2> $R/gpurun_out/${TAG}_trace.err
