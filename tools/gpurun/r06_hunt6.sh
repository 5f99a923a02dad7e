# usage: bash tools/gpurun/r06_hunt6.sh TAG N -- fresh C5 processes interleaved over three grouping configurations
# (adaptive default; fixed 32-set groups; fixed 1,024-set groups), N each, with a mismatch's call index recorded
TAG=$1; N=${2:-20}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in $(seq 1 $N); do
  for cfg in "adapt:" "g32:--set group_adapt=0 --group-sets 32" "g1024:--set group_adapt=0"; do
    name=${cfg%%:*}; opts=${cfg#*:}
    timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 64 --no-cpu-baseline \
      --no-profile --no-parity $opts > gpurun_out/${TAG}_${name}_r$rep.json 2> gpurun_out/${TAG}_${name}_r$rep.err
    r=$?; echo "$name $rep $r" >> gpurun_out/${TAG}_rc.txt; [ $r -le 1 ] || exit $r
  done
done
