# usage: bash tools/gpurun/r06_poison.sh TAG -- every fresh device / pinned buffer poisoned (BLSGPU_POISON=1): the GPU
# suite, the C5 stress test, C5 and C2 bench processes -- a kernel reading memory its run never wrote fails every time
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export BLSGPU_POISON=1
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
echo "suite $?" >> gpurun_out/${TAG}_rc.txt
for rep in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 16 --no-cpu-baseline \
    --no-profile > gpurun_out/${TAG}_C5_r$rep.json 2> gpurun_out/${TAG}_C5_r$rep.err
  r=$?; echo "C5 $rep $r" >> gpurun_out/${TAG}_rc.txt; [ $r -le 1 ] || exit $r
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_C2.json \
  2> gpurun_out/${TAG}_C2.err
echo "C2 $?" >> gpurun_out/${TAG}_rc.txt
