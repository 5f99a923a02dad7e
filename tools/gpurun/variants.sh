# usage: bash tools/gpurun/variants.sh TAG "lib1 lib2 ..." "inflight list"  -- GPU tests (default lib), then the
# C2 bench for every (library variant, in-flight depth) pair; a variant is lodestar_amd/variants/<name>.so
set -e
TAG=$1; LIBS=$2; LIST=$3; shift 3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for L in $LIBS; do
  for d in $LIST; do
    if [ "$L" = default ]; then P=""; else P=$GRAFT_REPO_ROOT/lodestar_amd/variants/$L.so; fi
    BLSGPU_LIB=$P timeout -k 10 200 python bench.py --inflight $d --no-cpu-baseline "$@" > gpurun_out/${TAG}_${L}_if$d.json 2> gpurun_out/${TAG}_${L}_if$d.err
  done
done
