# usage: bash tools/gpurun/r06_f.sh TAG LIB... -- interleaved A/B of library variants (BLSGPU_LIB) on the driver's C2
# command (3 rounds at 20 steps, 2 rounds at 100 steps); "base" = the in-tree library
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in "$@"; do
    L=lodestar_amd/libblsgpu.so; [ "$v" = base ] || L=lodestar_amd/variants/libv_$v.so
    BLSGPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
      > gpurun_out/${TAG}_${v}_20_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
for rep in 1 2; do
  for v in "$@"; do
    L=lodestar_amd/libblsgpu.so; [ "$v" = base ] || L=lodestar_amd/variants/libv_$v.so
    BLSGPU_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity \
      > gpurun_out/${TAG}_${v}_100_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
