# usage: bash tools/gpurun/r05_ad.sh TAG -- kernel timelines of isolated small calls (C5: 1,024 sets, 1% invalid,
# with its fallback; C1: 128 sets) on the current build
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in C5 C1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_$C -o run -- python3 $R/bench.py --config $C --steps 4 --warmup 1 --inflight 1 --no-cpu-baseline --no-parity --no-profile > $R/gpurun_out/${TAG}_$C.json 2> $R/gpurun_out/${TAG}_$C.err
done
