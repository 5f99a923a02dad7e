# usage: bash tools/gpurun/r06_n.sh TAG -- burst-ramp option sweep on the driver's C2 command (20 steps): for each
# option set, 3 interleaved rounds, then one kernel trace (the run structure of the window)
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
CFGS=("base:spec_gsm=0" "gsm:spec_gsm=1" "nolarge:spec_large=0,spec_gsm=0" "gsm_copy:spec_gsm=1,copy_stream=1"
      "nolarge_idle:spec_large=0,idle_wait_us=2000" "gsm_copy_idle:spec_gsm=1,copy_stream=1,idle_wait_us=2000"
      "copy:spec_gsm=0,copy_stream=1")
sets() { local o=""; IFS=',' read -ra kv <<< "$1"; for x in "${kv[@]}"; do o="$o --set $x"; done; echo $o; }
for rep in 1 2 3; do
  for c in "${CFGS[@]}"; do
    name=${c%%:*}; opts=$(sets ${c#*:})
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile $opts \
      > gpurun_out/${TAG}_${name}_r$rep.json 2>> gpurun_out/${TAG}.err
  done
done
cd /tmp && export TMPDIR=/tmp
for c in "${CFGS[@]}"; do
  name=${c%%:*}; opts=$(sets ${c#*:})
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_tr_${name} -o run -- python3 \
    $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-profile $opts \
    > $R/gpurun_out/${TAG}_tr_${name}.json 2>> $R/gpurun_out/${TAG}.err
done
