# usage: bash tools/gpurun/r05_at.sh TAG -- after the coop edge change: mid-size / parity / option tests, then a kernel
# trace of isolated calls at 128 / 1,024 / 4,096 sets (critical path of small and mid-size runs)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_midsize.py tests/test_gpu_options.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for s in 128 1024 4096; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tr$s -o run -- python3 -u tools/latency_curve.py --sizes $s --reps 3 --variants "base:" > gpurun_out/${TAG}_tr$s.log 2>&1
done
