# usage: bash tools/gpurun/r05_ai.sh TAG -- kernel + memory-copy trace of the driver's C2 command (run formation,
# host-to-device staging of merged runs), and the isolated-call host overhead per config
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 $R/tools/host_overhead.py --configs C2,C1,C5,C3 --out $R/gpurun_out/${TAG}_host.json > $R/gpurun_out/${TAG}_host.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $R/gpurun_out/${TAG}_trace.json 2> $R/gpurun_out/${TAG}_trace.err
