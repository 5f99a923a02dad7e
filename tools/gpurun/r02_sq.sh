# usage: bash tools/gpurun/r02_sq.sh TAG  -- one rocprofv3 PMC pass of 8 SQ counters (issue / wait / active cycles)
# over serial 16,384-set C2 launches, kernel trace only
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --inflight 1 --slots 1 --no-profile --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq.log 2>&1
