# usage: bash tools/gpurun/r06_j.sh TAG -- the urgent tests (burst linger) and options; blocking_sync 1 / 0 on the
# driver's C2 command (3 interleaved rounds at 20 steps, 1 at 100; host CPU seconds per million sets in each line);
# then r06_i.sh (spec_large on C5 / C1 / C4, idle_wait_us on C2)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max > gpurun_out/${TAG}_cgroup.txt 2>&1 || true
nproc >> gpurun_out/${TAG}_cgroup.txt 2>&1 || true
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_urgent.py tests/test_gpu_options.py -v -s --timeout 240 \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || rc=$?
[ $rc -le 1 ] || exit $rc
for rep in 1 2 3; do
  for bs in 1 0; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --set blocking_sync=$bs > gpurun_out/${TAG}_bs${bs}_20_r$rep.json 2>> gpurun_out/${TAG}_bs.err
  done
done
for bs in 1 0; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
    --set blocking_sync=$bs > gpurun_out/${TAG}_bs${bs}_100.json 2>> gpurun_out/${TAG}_bs.err
done
bash tools/gpurun/r06_i.sh ${TAG}i
