# usage: bash tools/gpurun/r05_ar.sh TAG -- isolated p50 curve around the cooperative Miller threshold (coop_max 512
# default vs 256 / 384), valid calls and 1%-invalid C5-shaped calls
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/latency_curve.py --sizes 128,256,384,512,768,1024 --reps 9 --variants "c512:;c384:coop_max=384;c256:coop_max=256" --out gpurun_out/${TAG}_curve.json > gpurun_out/${TAG}_curve.log 2>&1
timeout -k 10 400 python -u tools/latency_curve.py --sizes 256,384,512,768,1024 --reps 9 --invalid 0.01 --jobs3 --variants "c512:;c384:coop_max=384;c256:coop_max=256" --out gpurun_out/${TAG}_curve_inv.json > gpurun_out/${TAG}_curve_inv.log 2>&1
