set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/mad_chain > gpurun_out/r02_mad_chain.json 2>&1
bash tools/gpurun/r02_tb.sh r02p
