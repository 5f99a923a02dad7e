# usage: bash tools/gpurun/r05_o.sh TAG -- six-lane check parity tests; C5 under load check6 on/off
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_midsize.py -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
i=0
for V in "" "--set fb_check6=0"; do
  i=$((i+1))
  echo "$V" > gpurun_out/${TAG}_C5_v$i.args
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 --no-cpu-baseline --no-parity $V > gpurun_out/${TAG}_C5_v$i.json 2> gpurun_out/${TAG}_C5_v$i.err
done
