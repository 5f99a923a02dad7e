# usage: bash tools/gpurun/r06_r.sh TAG -- C5 and C4 over longer timed windows (C5 2,000 steps ~3 s, C4 200 steps ~3 s
# instead of 400 / 40): run-to-run spread, C5 with group_adapt 1 / 0 interleaved (3 rounds), C4 3 rounds
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  for a in 1 0; do
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline \
      --no-parity --no-profile --set group_adapt=$a > gpurun_out/${TAG}_C5_a${a}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
  timeout -k 10 200 python -u bench.py --config C4 --inflight 8 --steps 200 --warmup 16 --no-cpu-baseline \
    --no-parity --no-profile > gpurun_out/${TAG}_C4_r$rep.json 2>> gpurun_out/${TAG}.err
done
