# usage: bash tools/gpurun/r06_v.sh TAG -- spurious batch-group failures: all-valid C2 calls (expected all 1) with
# one-set groups (group_sets 1, group_adapt 0: every set's own equation, a failed one answers false directly), and the
# driver's C2 command's fallback count; the C5 stress test
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --inflight 8 --no-cpu-baseline --no-parity --no-profile \
    --group-sets 1 --set group_adapt=0 > gpurun_out/${TAG}_g1_r$rep.json 2> gpurun_out/${TAG}_g1_r$rep.err
  echo "g1 rep $rep rc $?" >> gpurun_out/${TAG}_rc.txt
done
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
    > gpurun_out/${TAG}_c2_r$rep.json 2> gpurun_out/${TAG}_c2_r$rep.err
  echo "c2 rep $rep rc $?" >> gpurun_out/${TAG}_rc.txt
done
