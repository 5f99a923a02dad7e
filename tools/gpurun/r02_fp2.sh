set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/fp2_rate > gpurun_out/r02s4_fp2_rate.json 2>&1
bash tools/gpurun/r02_sweep3.sh r02s4_sw4 "-|--steps 300" "libblsgpu_wpe2.so|--steps 300"
