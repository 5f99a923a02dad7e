# usage: bash tools/gpurun/r05_fbtrace.sh TAG -- kernel traces of the 1%-invalid (fallback) path: an isolated 1024-set
# call and a loaded run (32 in flight), C5 job shape, single-key sets
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_iso -o run -- \
  python3 $R/tools/latency_curve.py --sizes 1024 --variants 'base:' --invalid 0.01 --jobs3 --reps 3 > $R/gpurun_out/${TAG}_iso.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_load -o run -- \
  python3 $R/tools/latency_curve.py --sizes 1024 --variants 'base:' --invalid 0.01 --jobs3 --reps 1 --load-steps 64 > $R/gpurun_out/${TAG}_load.log 2>&1
