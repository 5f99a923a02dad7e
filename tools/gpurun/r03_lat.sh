# usage: bash tools/gpurun/r03_lat.sh TAG [CONFIG...] -- kernel traces of serial calls (default C1 and C3, one call
# in flight):
# per-kernel durations on the critical path of an isolated call
set -e
TAG=$1; shift
CFGS=${@:-C1 C3}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_$C.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_$C.log
done
