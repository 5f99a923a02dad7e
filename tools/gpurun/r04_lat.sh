# usage: bash tools/gpurun/r04_lat.sh TAG "args1|args2|..."  -- serial 16k-call latency (bench --inflight 1) per
# argument set (e.g. "--miller-lanes 1|--miller-lanes 2"), rocprofv3 kernel trace of each
set -e
TAG=$1; IFS='|' read -ra SETS <<< "$2"
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
k=0
for A in "${SETS[@]}"; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_lat$k -o run -- python3 $GRAFT_REPO_ROOT/bench.py --inflight 1 --steps 10 --warmup 2 --no-parity --no-cpu-baseline $A > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_lat$k.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_lat$k.err )
  echo "$k: $A" >> gpurun_out/${TAG}_lat_index.txt
  k=$((k+1))
done
