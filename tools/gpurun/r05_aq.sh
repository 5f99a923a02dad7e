# usage: bash tools/gpurun/r05_aq.sh TAG -- C4 (and C2 20-step) on the current build vs the build of f52a7c8
# (libblsgpu_old.so: before the host run-formation changes), three interleaved rounds
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for r in a b c; do
  for L in cur old; do
    LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu.so
    [ $L = old ] && LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_old.so
    i=$((i+1)); echo "C4 $L" > gpurun_out/${TAG}_$i.args
    BLSGPU_LIB=$LIB timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
    i=$((i+1)); echo "C2 $L" > gpurun_out/${TAG}_$i.args
    BLSGPU_LIB=$LIB timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
