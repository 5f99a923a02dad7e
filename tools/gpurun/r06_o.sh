# usage: bash tools/gpurun/r06_o.sh TAG -- kernel traces of isolated 1-set and 128-set calls (the latency floor)
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for n in 1 128; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/${TAG}_s$n -o run -- \
    python3 $R/tools/latency_curve.py --sizes $n --reps 8 --variants "base:" --out $R/gpurun_out/${TAG}_s$n.json \
    > $R/gpurun_out/${TAG}_s$n.log 2>&1
done
