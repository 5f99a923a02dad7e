# usage: bash tools/gpurun/r04_sweep.sh TAG REPS "args1|args2|..." -- driver-command (20 steps, 5 warmup) C2 throughput
# per bench argument set, interleaved over REPS rounds
TAG=$1; REPS=$2; IFS='|' read -ra SETS <<< "$3"
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  k=0
  for A in "${SETS[@]}"; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity $A \
      > gpurun_out/${TAG}_${k}_${r}.json 2> gpurun_out/${TAG}_${k}_${r}.err || { echo "[$A] rep $r failed"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '|', d['value'], d.get('p50_batch_latency_ms'), d['config'].get('pipeline_runs_timed'))" gpurun_out/${TAG}_${k}_${r}.json "$A"
    k=$((k+1))
  done
done
