# usage: bash tools/gpurun/r06_k.sh TAG -- urgent lane on HIP's high-priority queues with the pipeline at normal
# priority (urgent_isolate 2, pipeline_prio 0) vs the default lane: urgent latency alone and under a 200-step C2 flood
# (2 rounds each), and the driver's C2 command with and without pipeline priorities (3 interleaved rounds)
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "1 1" "2 0"; do
    set -- $cfg
    timeout -k 10 240 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --urgent-every-ms 10 --set urgent_isolate=$1 --set pipeline_prio=$2 > gpurun_out/${TAG}_lat_i$1_p$2_r$rep.json \
      2>> gpurun_out/${TAG}_lat.err
  done
done
for rep in 1 2 3; do
  for pp in 1 0; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
      --set pipeline_prio=$pp > gpurun_out/${TAG}_pp${pp}_r$rep.json 2>> gpurun_out/${TAG}_pp.err
  done
done
