# usage: bash tools/gpurun/r05_bb.sh TAG -- kernel trace of the driver's command with alone_msm
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 $R/bench.py --gpus 1 --warmup 5 --steps 20 --no-cpu-baseline --no-parity --set alone_msm=1 > $R/gpurun_out/${TAG}_trace.json 2> $R/gpurun_out/${TAG}_trace.err
