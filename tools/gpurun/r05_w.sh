# usage: bash tools/gpurun/r05_w.sh TAG -- lane-pair Miller accumulation (miller_lanes 3): parity (chunk forms,
# mid-size forms, units) and C2 A/B against the default forms, 20 and 100 steps
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_midsize.py -x -v --timeout 250 --timeout-method thread -k "chunk_forms or forms_agree or units_recompute or 8192" > gpurun_out/${TAG}_tests.log 2>&1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
$B --miller-lanes 3 > gpurun_out/${TAG}_m3a.json 2> gpurun_out/${TAG}_m3a.err
$B --no-parity > gpurun_out/${TAG}_m0a.json 2> gpurun_out/${TAG}_m0a.err
$B --no-parity --miller-lanes 3 > gpurun_out/${TAG}_m3b.json 2> gpurun_out/${TAG}_m3b.err
$B --no-parity > gpurun_out/${TAG}_m0b.json 2> gpurun_out/${TAG}_m0b.err
B="timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity"
$B --miller-lanes 3 > gpurun_out/${TAG}_m3c.json 2> gpurun_out/${TAG}_m3c.err
$B > gpurun_out/${TAG}_m0c.json 2> gpurun_out/${TAG}_m0c.err
