# usage: bash tools/gpurun/r04_sq.sh TAG  -- VALU-utilisation evidence for the driver's command (C2, 20 steps): rocprofv3
# PMC passes (kernel trace only, one counter group per pass, <= 8 SQ + 2 GRBM counters), plus the list of counters the
# box offers.
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_avail.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq1.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_sq1.err
