# usage: bash tools/gpurun/r06_valid.sh TAG N -- the GPU suite, one C5 evidence line (2,000 steps, parity leg), then N
# fresh C5 processes (1,000 steps each), all on the library's defaults
TAG=$1; N=${2:-40}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config C5 --inflight 32 --steps 2000 > gpurun_out/${TAG}_C5.json 2> gpurun_out/${TAG}_C5.err || exit $?
for rep in $(seq 1 $N); do
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 1000 --warmup 64 \
    --no-cpu-baseline --no-profile --no-parity > gpurun_out/${TAG}_r$rep.json 2> gpurun_out/${TAG}_r$rep.err
  r=$?; echo "$rep $r" >> gpurun_out/${TAG}_rc.txt; [ $r -le 1 ] || exit $r
done
