# usage: bash tools/gpurun/r05_v.sh TAG -- lane-pair Miller lines: parity (line tests, mid-size forms) and C2 A/B
# lines_lanes 2 (pairs) vs 1 (one lane)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_midsize.py -x -v --timeout 250 --timeout-method thread -k "lines or 8192" > gpurun_out/${TAG}_tests.log 2>&1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
$B --lines-lanes 2 > gpurun_out/${TAG}_l2a.json 2> gpurun_out/${TAG}_l2a.err
$B --no-parity > gpurun_out/${TAG}_l1a.json 2> gpurun_out/${TAG}_l1a.err
$B --no-parity --lines-lanes 2 > gpurun_out/${TAG}_l2b.json 2> gpurun_out/${TAG}_l2b.err
$B --no-parity > gpurun_out/${TAG}_l1b.json 2> gpurun_out/${TAG}_l1b.err
