# usage: bash tools/gpurun/r05_be.sh TAG -- stream priorities off (BLSGPU_STREAM_PRIO=0 build, BLSGPU_LIB) against the
# product build: the driver's command five rounds interleaved, then 100 steps each
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="--gpus 1 --warmup 5 --no-cpu-baseline --no-parity"
NP=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_noprio.so
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py $B --steps 20 > gpurun_out/${TAG}_base_$i.json 2>/dev/null
  BLSGPU_LIB=$NP timeout -k 10 200 python -u bench.py $B --steps 20 > gpurun_out/${TAG}_np_$i.json 2>/dev/null
done
timeout -k 10 200 python -u bench.py $B --steps 100 > gpurun_out/${TAG}_base_100.json 2>/dev/null
BLSGPU_LIB=$NP timeout -k 10 200 python -u bench.py $B --steps 100 > gpurun_out/${TAG}_np_100.json 2>/dev/null
