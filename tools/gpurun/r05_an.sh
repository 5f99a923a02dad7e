# usage: bash tools/gpurun/r05_an.sh TAG -- the driver's 20-step C2 burst: idle-device merge wait and the input copy off
# the signature stream, three interleaved rounds; 100 steps once each
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for r in a b c; do
  for A in "" "--idle-wait-us 300" "--idle-wait-us 300 --set copy_stream=1" "--set copy_stream=1"; do
    i=$((i+1)); echo "20 $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
for A in "" "--idle-wait-us 300" "--idle-wait-us 300 --set copy_stream=1"; do
  i=$((i+1)); echo "100 $A" > gpurun_out/${TAG}_$i.args
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
done
