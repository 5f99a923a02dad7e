# usage: bash tools/gpurun/r05_i.sh TAG -- acc6 parity tests, latency curve acc6 vs acc2, inline-products A/B on C2
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_midsize.py tests/test_gpu_parity.py -x -v --timeout 250 --timeout-method thread -k "forms or chunk or one_percent" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u tools/latency_curve.py --sizes 1024,2048,4096,8192,16384,32768 --pool 32768 \
  --variants "acc6:;acc2:acc6_max=0;acc6nc:coop_max=0;acc6all:acc6_max=100000" --load-steps 100 \
  --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C2_def$r.json 2> gpurun_out/${TAG}_C2_def$r.err
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_inl.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C2_inl$r.json 2> gpurun_out/${TAG}_C2_inl$r.err
done
