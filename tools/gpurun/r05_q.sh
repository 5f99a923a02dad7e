# usage: bash tools/gpurun/r05_q.sh TAG -- MSM with inlined products (variant lib) vs default: C2 x2 each
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_def$r.json 2> gpurun_out/${TAG}_def$r.err
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_msminl.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_inl$r.json 2> gpurun_out/${TAG}_inl$r.err
done
