# usage: bash tools/gpurun/r04_pmc.sh TAG  -- HBM-traffic PMC passes over the driver's command (C2, 20 steps, 5 warmup),
# one counter per pass, kernel trace only (no sys/runtime trace), the program directly after --
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
