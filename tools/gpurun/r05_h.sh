# usage: bash tools/gpurun/r05_h.sh TAG -- kernel traces of isolated 128 / 1024 / 2048-set calls (defaults)
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for N in 128 1024 2048; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_n$N -o run -- \
  python3 $R/tools/latency_curve.py --sizes $N --variants 'base:' --reps 2 --pool $N > $R/gpurun_out/${TAG}_n$N.log 2>&1
done
