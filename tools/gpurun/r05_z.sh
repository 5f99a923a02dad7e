# usage: bash tools/gpurun/r05_z.sh TAG -- MSM bucket pass on lane pairs (k_msm_bucket2) vs one lane per bucket
# (libblsgpu_mp0.so), and lane-pair Miller lines: parity (MSM forms) + C2 A/B at 20 and 100 steps
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_midsize.py -x -v --timeout 250 --timeout-method thread -k "msm or slice or 8192 or 4096 or exceptional" > gpurun_out/${TAG}_tests.log 2>&1
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity"
for r in a b; do
  $B > gpurun_out/${TAG}_v1$r.json 2> gpurun_out/${TAG}_v1$r.err
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_mp0.so $B > gpurun_out/${TAG}_v2$r.json 2> gpurun_out/${TAG}_v2$r.err
  $B --lines-lanes 2 > gpurun_out/${TAG}_v3$r.json 2> gpurun_out/${TAG}_v3$r.err
done
B="timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity"
$B > gpurun_out/${TAG}_v1c.json 2> gpurun_out/${TAG}_v1c.err
BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/libblsgpu_mp0.so $B > gpurun_out/${TAG}_v2c.json 2> gpurun_out/${TAG}_v2c.err
$B --lines-lanes 2 > gpurun_out/${TAG}_v3c.json 2> gpurun_out/${TAG}_v3c.err
