# usage: bash tools/gpurun/r05_final2.sh TAG -- round-5 final bench lines: C2 (the driver's command, with parity and
# cpu_baseline), C1 / C3 / C5 at 32 calls in flight, C4 (32,768 aggregate sets, 8 in flight), each with its parity leg
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_C2.json 2> gpurun_out/${TAG}_C2.err
timeout -k 10 300 python -u bench.py --config C1 --inflight 32 --steps 1000 --warmup 64 > gpurun_out/${TAG}_C1.json 2> gpurun_out/${TAG}_C1.err
timeout -k 10 300 python -u bench.py --config C3 --inflight 32 --steps 300 --warmup 32 > gpurun_out/${TAG}_C3.json 2> gpurun_out/${TAG}_C3.err
timeout -k 10 300 python -u bench.py --config C5 --inflight 32 --steps 400 --warmup 32 > gpurun_out/${TAG}_C5.json 2> gpurun_out/${TAG}_C5.err
timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 40 --warmup 8 > gpurun_out/${TAG}_C4.json 2> gpurun_out/${TAG}_C4.err
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C2_100.json 2> gpurun_out/${TAG}_C2_100.err
timeout -k 10 300 python -u tools/latency_curve.py --sizes 128,256,512,1024,2048,4096,8192,16384 --variants "final:" --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
