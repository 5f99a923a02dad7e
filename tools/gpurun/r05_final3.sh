# usage: bash tools/gpurun/r05_final3.sh TAG -- evidence + bench lines on the current build in one call
# (r05_final1.sh: full GPU suite, smoke, driver-command trace / PMC / SQ passes; r05_final2.sh: C1-C5 lines, curve)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
md5sum lodestar_amd/libblsgpu.so > gpurun_out/${TAG}_md5.txt
bash tools/gpurun/r05_final1.sh $TAG
bash tools/gpurun/r05_final2.sh $TAG
