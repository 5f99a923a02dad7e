# usage: bash tools/gpurun/r06_w.sh TAG -- after the single-clean-job re-check: the whole GPU suite (C5 stress test
# included), then fresh C5 bench processes (parity leg, 64-round warm-up) and C2 at 100 steps, each line carrying the
# runtime's spurious_groups count
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rc=0
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for rep in 1 2 3 4 5 6; do
  timeout -k 10 200 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 64 --no-cpu-baseline \
    --no-profile > gpurun_out/${TAG}_C5_r$rep.json 2> gpurun_out/${TAG}_C5_r$rep.err
  r=$?; echo "C5 rep $rep rc $r" >> gpurun_out/${TAG}_rc.txt; [ $r -le 1 ] || exit $r
done
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
    > gpurun_out/${TAG}_C2_r$rep.json 2> gpurun_out/${TAG}_C2_r$rep.err
  r=$?; echo "C2 rep $rep rc $r" >> gpurun_out/${TAG}_rc.txt; [ $r -le 1 ] || exit $r
done
