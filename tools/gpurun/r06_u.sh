# usage: bash tools/gpurun/r06_u.sh TAG N -- N fresh bench.py C5 processes with the parity leg and a 64-round warm-up
# (the command that once returned false for a valid job, r06s): each stops at its first mismatch with the call's stats
TAG=$1; N=${2:-8}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in $(seq 1 $N); do
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 200 --warmup 64 --no-cpu-baseline \
    --no-profile > gpurun_out/${TAG}_C5_r$rep.json 2> gpurun_out/${TAG}_C5_r$rep.err
  rc=$?
  echo "rep $rep rc $rc" >> gpurun_out/${TAG}_rc.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
