# usage: bash tools/gpurun/evidence.sh TAG -- evidence of the driver's command (C2, 20 steps, 5 warmup) on the
# current build: kernel trace + stats, FETCH_SIZE / WRITE_SIZE PMC passes, SQ counter pass (each its own run, kernel
# trace only, the program directly after --)
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
A="--gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 $R/bench.py $A --no-cpu-baseline --no-parity > $R/gpurun_out/${TAG}_trace.json 2> $R/gpurun_out/${TAG}_trace.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/${TAG}_pmc_$C -o run -- python3 $R/bench.py $A --no-cpu-baseline --no-parity --no-profile > $R/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/${TAG}_sq1 -o run -- python3 $R/bench.py $A --no-cpu-baseline --no-parity > $R/gpurun_out/${TAG}_sq1.json 2> $R/gpurun_out/${TAG}_sq1.err
