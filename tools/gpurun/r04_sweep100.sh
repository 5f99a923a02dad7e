# usage: bash tools/gpurun/r04_sweep100.sh TAG REPS "args1|args2" -- 100-step C2 throughput per bench argument set
TAG=$1; REPS=$2; IFS='|' read -ra SETS <<< "$3"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in $(seq 1 $REPS); do k=0; for A in "${SETS[@]}"; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_${k}_${r}.json 2> gpurun_out/${TAG}_${k}_${r}.err || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '|', d['value'])" gpurun_out/${TAG}_${k}_${r}.json "$A"; k=$((k+1)); done; done
