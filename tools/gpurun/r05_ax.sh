# usage: bash tools/gpurun/r05_ax.sh TAG -- base vs ramp_swap + copy_stream at the driver's 20 steps, five rounds
# interleaved, then a kernel trace of the swapped configuration
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
B="--gpus 1 --warmup 5 --steps 20 --no-cpu-baseline --no-parity"
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py $B > gpurun_out/${TAG}_base_$i.json 2>/dev/null
  timeout -k 10 200 python -u bench.py $B --set ramp_swap=1 --set copy_stream=1 > gpurun_out/${TAG}_sc_$i.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 $R/bench.py $B --set ramp_swap=1 --set copy_stream=1 > $R/gpurun_out/${TAG}_trace.json 2> $R/gpurun_out/${TAG}_trace.err
