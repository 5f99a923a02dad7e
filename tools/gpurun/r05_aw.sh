# usage: bash tools/gpurun/r05_aw.sh TAG -- ramp_swap A/B on the driver's command (C2, 20 steps) and at 100 steps,
# interleaved: base / ramp_swap / ramp_swap + copy_stream, three rounds at 20 steps, one at 100
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--gpus 1 --warmup 5 --no-cpu-baseline --no-parity"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py $B --steps 20 > gpurun_out/${TAG}_base_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py $B --steps 20 --set ramp_swap=1 > gpurun_out/${TAG}_swap_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py $B --steps 20 --set ramp_swap=1 --set copy_stream=1 > gpurun_out/${TAG}_swapcopy_$i.json 2>/dev/null
done
timeout -k 10 200 python -u bench.py $B --steps 100 > gpurun_out/${TAG}_base_100.json 2>/dev/null
timeout -k 10 200 python -u bench.py $B --steps 100 --set ramp_swap=1 > gpurun_out/${TAG}_swap_100.json 2>/dev/null
