# usage: bash tools/gpurun/r05_aj.sh TAG -- the group stage on the message stream (tail_on_msg) and the input copy
# off the signature stream (copy_stream): parity (pipeline, configs) + C2 at 20 (x3) and 100 steps, C1 / C5
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --set tail_on_msg=1 --set copy_stream=1 > gpurun_out/${TAG}_par_c2.json 2> gpurun_out/${TAG}_par_c2.err
timeout -k 10 300 python -u bench.py --config C5 --steps 100 --warmup 32 --no-cpu-baseline --set tail_on_msg=1 --set copy_stream=1 > gpurun_out/${TAG}_par_c5.json 2> gpurun_out/${TAG}_par_c5.err
i=0
for r in a b c; do
  for A in "" "--set tail_on_msg=1" "--set copy_stream=1" "--set tail_on_msg=1 --set copy_stream=1"; do
    i=$((i+1)); echo "20 $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
for A in "" "--set tail_on_msg=1 --set copy_stream=1"; do
  i=$((i+1)); echo "100 $A" > gpurun_out/${TAG}_$i.args
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  for C in C1 C5; do
    i=$((i+1)); echo "$C $A" > gpurun_out/${TAG}_$i.args
    timeout -k 10 300 python -u bench.py --config $C --steps 300 --warmup 32 --no-cpu-baseline --no-parity $A > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
  done
done
