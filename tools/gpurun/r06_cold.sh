# usage: bash tools/gpurun/r06_cold.sh TAG N -- N cold C5 contexts (fresh context, device-signed variants, one round of
# 32 calls), mismatches diagnosed against the CPU oracle (signer vs verifier)
TAG=$1; N=${2:-40}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
C5_COLD_ROUNDS=$N timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_stress.py -k cold -v -s --timeout 850 \
  --timeout-method thread > gpurun_out/${TAG}_cold.log 2>&1
echo "cold $?" > gpurun_out/${TAG}_rc.txt
