# usage: bash tools/gpurun/r06_i.sh TAG -- spec_large on / off on C5, C1, C4 (r06_e.sh, 3 interleaved rounds), then
# the burst ramp: idle_wait_us 0 / 500 / 2000 on the driver's C2 command, 3 interleaved rounds
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpurun/r06_e.sh ${TAG}s
for rep in 1 2 3; do
  for iw in 0 500 2000; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --idle-wait-us $iw > gpurun_out/${TAG}_iw${iw}_r$rep.json 2>> gpurun_out/${TAG}_iw.err
  done
done
