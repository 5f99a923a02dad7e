# usage: bash tools/gpurun/r06_final.sh TAG -- round-6 evidence on the final library, one call:
#  1. the driver's command under rocprofv3: kernel trace + stats, FETCH_SIZE / WRITE_SIZE PMC passes, SQ counter pass
#     (r05_evidence.sh); the PMC passes folded into profiles/r06_pmc_traffic.json on the box, which the bench lines read
#  2. bench lines with parity and cpu_baseline: C2 (the driver's command), C2 at 100 steps, C1 / C3 / C5 at 32 calls in
#     flight, C4 at 8 (timed windows of ~1-3 s: C1 5,000 steps, C3 3,000, C5 2,000, C4 200); the isolated latency curve from 1 set; the 8-context host-capacity mode; the urgent probe
#  3. a kernel trace of the urgent probe under the flood (tools/urgent_wait.py)
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/gpurun/evidence.sh ${TAG}e
cd $R
python tools/pmc_to_json.py gpurun_out/${TAG}e profiles/r06_pmc_traffic.json > gpurun_out/${TAG}_pmc_fold.log 2>&1
cp profiles/r06_pmc_traffic.json gpurun_out/${TAG}_pmc_traffic.json
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_C2.json 2> gpurun_out/${TAG}_C2.err
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_C2_100.json 2> gpurun_out/${TAG}_C2_100.err
timeout -k 10 300 python -u bench.py --config C1 --inflight 32 --steps 5000 --warmup 64 > gpurun_out/${TAG}_C1.json 2> gpurun_out/${TAG}_C1.err
timeout -k 10 300 python -u bench.py --config C3 --inflight 32 --steps 3000 --warmup 32 > gpurun_out/${TAG}_C3.json 2> gpurun_out/${TAG}_C3.err
timeout -k 10 300 python -u bench.py --config C5 --inflight 32 --steps 2000 --warmup 32 > gpurun_out/${TAG}_C5.json 2> gpurun_out/${TAG}_C5.err
timeout -k 10 300 python -u bench.py --config C4 --inflight 8 --steps 200 --warmup 8 > gpurun_out/${TAG}_C4.json 2> gpurun_out/${TAG}_C4.err
timeout -k 10 300 python -u tools/latency_curve.py --sizes 1,3,16,32,128,256,512,1024,2048,4096,8192,16384 \
  --variants "final:" --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 8 --devices-same 0 --inflight 8 --steps 20 --warmup 3 --no-cpu-baseline \
  --no-parity > gpurun_out/${TAG}_host8.json 2> gpurun_out/${TAG}_host8.err
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity --no-profile \
  --urgent-every-ms 10 > gpurun_out/${TAG}_urgent.json 2> gpurun_out/${TAG}_urgent.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_utrace -o run -- python3 \
  $R/bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-parity --no-profile --urgent-every-ms 10 \
  > $R/gpurun_out/${TAG}_utrace.json 2> $R/gpurun_out/${TAG}_utrace.err
