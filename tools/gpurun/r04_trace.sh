# usage: bash tools/gpurun/r04_trace.sh TAG [bench args]  -- rocprofv3 kernel trace + stats of the driver's command
# (default: C2, 20 steps, 5 warmup), the program directly after --
TAG=$1; shift
ARGS=${@:-"--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity"}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace.err
