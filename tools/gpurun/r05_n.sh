# usage: bash tools/gpurun/r05_n.sh TAG -- sweep: C5 direct threshold, C1/C3/C2 pipeline depth
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
run() {  # config steps warmup args...
  i=$((i+1)); C=$1; S=$2; W=$3; shift 3
  echo "$C $*" > gpurun_out/${TAG}_v$i.args
  timeout -k 10 200 python -u bench.py --config $C --inflight 32 --steps $S --warmup $W --no-cpu-baseline --no-parity "$@" > gpurun_out/${TAG}_v$i.json 2> gpurun_out/${TAG}_v$i.err
}
run C5 400 32 --set fb_direct_min=512
run C5 400 32
run C1 1000 64 --pipeline-depth 2
run C1 1000 64
run C1 1000 64 --pipeline-depth 4
run C3 300 32 --pipeline-depth 2
run C3 300 32
run C2 20 5 --pipeline-depth 2
run C2 20 5
