# usage: bash tools/gpurun/r04_iso.sh TAG [sets]  -- per-kernel isolation profile: one call of SETS (default 131072) C2
# sets per step, every branch of the run on one stream (option "serial"), so each kernel runs alone on the chip;
# rocprofv3 kernel trace + stats.
set -e
TAG=$1; SETS=${2:-131072}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_iso -o run -- python3 $GRAFT_REPO_ROOT/bench.py --sets $SETS --inflight 1 --steps 3 --warmup 1 --serial --no-parity --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_iso.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_iso.err
