# usage: bash tools/gpurun/r06_e.sh TAG -- verdict r5 #6: five interleaved rounds of spec_large on / off on C5, C4 and C1
# (bench lines without parity / cpu baseline; parity is covered by the tests and the final lines)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  for sl in 1 0; do
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline \
      --no-parity --no-profile --set spec_large=$sl > gpurun_out/${TAG}_C5_sl${sl}_r$rep.json 2>> gpurun_out/${TAG}.err
    timeout -k 10 200 python -u bench.py --config C1 --inflight 32 --steps 1000 --warmup 64 --no-cpu-baseline \
      --no-parity --no-profile --set spec_large=$sl > gpurun_out/${TAG}_C1_sl${sl}_r$rep.json 2>> gpurun_out/${TAG}.err
    timeout -k 10 240 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline \
      --no-parity --no-profile --set spec_large=$sl > gpurun_out/${TAG}_C4_sl${sl}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
