# usage: bash tools/gpurun/r02_pmc.sh TAG  -- HBM traffic per kernel: two rocprofv3 PMC passes (FETCH_SIZE, then
# WRITE_SIZE; TCC has 4 counters and they need 3 + 2), kernel trace only, over serial 16,384-set C2 launches;
# fold with: python tools/pmc_to_json.py gpurun_out/TAG profiles/TAG_pmc_traffic.json
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --inflight 1 --slots 1 --no-profile --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_$C.log 2>&1
done
