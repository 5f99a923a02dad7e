# usage: bash tools/gpurun/r02_variant.sh TAG LIB [K...]  -- bench lines of a library variant over miller_k
set -e
TAG=$1; LIBV=$2; shift 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
for K in "$@"; do
  BLSGPU_LIB=$GRAFT_REPO_ROOT/lodestar_amd/$LIBV timeout -k 10 200 python bench.py --no-cpu-baseline --miller-k $K > gpurun_out/${TAG}_k$K.json 2> gpurun_out/${TAG}_k$K.err
done
