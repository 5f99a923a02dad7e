# usage: bash tools/gpurun/r05_y.sh TAG -- per-kernel SQ counters and kernel traces of C2 (driver's command) with the
# lane-pair accumulation on / off (miller_pairs), lane-pair MSM bucket pass in both
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
A="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity"
for P in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_trace_p$P -o run -- python3 $R/bench.py $A --set miller_pairs=$P > $R/gpurun_out/${TAG}_trace_p$P.json 2> $R/gpurun_out/${TAG}_trace_p$P.err
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/${TAG}_sq_p$P -o run -- python3 $R/bench.py $A --set miller_pairs=$P > $R/gpurun_out/${TAG}_sq_p$P.json 2> $R/gpurun_out/${TAG}_sq_p$P.err
done
