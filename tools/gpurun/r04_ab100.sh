# usage: bash tools/gpurun/r04_ab100.sh TAG REPS "lib1 lib2" -- 100-step C2 throughput of library variants
TAG=$1; REPS=$2; LIBS=$3
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in $(seq 1 $REPS); do for L in $LIBS; do
  if [ "$L" = default ]; then P=""; else P=$GRAFT_REPO_ROOT/lodestar_amd/variants/$L.so; fi
  BLSGPU_LIB=$P timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_${L}_$r.json 2> gpurun_out/${TAG}_${L}_$r.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'])" gpurun_out/${TAG}_${L}_$r.json $L $r
done; done
