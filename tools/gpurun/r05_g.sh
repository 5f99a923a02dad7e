# usage: bash tools/gpurun/r05_g.sh TAG -- full GPU tests, smoke, C2 default bench, C4 bench on one device
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_C2.json 2> gpurun_out/${TAG}_C2.err
timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C4.json 2> gpurun_out/${TAG}_C4.err
