# usage: bash tools/gpurun/r06_l.sh TAG -- the whole GPU suite (group_adapt on by default now), then C5 (1% invalid,
# 32 calls in flight) with adaptive group sizes vs fixed 1024 / 64 / 16, 2 interleaved rounds, and the driver's C2
# command with group_adapt 1 / 0 (all valid: must be equal)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for cfg in "1 1024" "0 1024" "0 64" "0 16"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline \
      --no-parity --set group_adapt=$1 --group-sets $2 > gpurun_out/${TAG}_C5_a$1_g$2_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
for rep in 1 2; do
  for a in 1 0; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --set group_adapt=$a > gpurun_out/${TAG}_C2_a${a}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
