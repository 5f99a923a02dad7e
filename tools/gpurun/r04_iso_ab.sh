# usage: bash tools/gpurun/r04_iso_ab.sh TAG SETS "lib1 lib2 ..."  -- the isolation profile (r04_iso.sh) for each
# library variant (default = the in-tree build, else lodestar_amd/variants/<name>.so), then a 20-step C2 bench each
# each variant runs under its own time limit; a failing one does not stop the rest
TAG=$1; SETS=$2; LIBS=$3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in $LIBS; do
  if [ "$L" = default ]; then P=""; else P=$GRAFT_REPO_ROOT/lodestar_amd/variants/$L.so; fi
  ( cd /tmp && export TMPDIR=/tmp && BLSGPU_LIB=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${L}_iso -o run -- python3 $GRAFT_REPO_ROOT/bench.py --sets $SETS --inflight 1 --steps 3 --warmup 1 --serial --no-parity --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${L}_iso.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_${L}_iso.err )
done
for L in $LIBS; do
  if [ "$L" = default ]; then P=""; else P=$GRAFT_REPO_ROOT/lodestar_amd/variants/$L.so; fi
  BLSGPU_LIB=$P timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_${L}_c2.json 2> gpurun_out/${TAG}_${L}_c2.err
done
