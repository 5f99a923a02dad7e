# usage: bash tools/gpurun/r06_d2.sh TAG -- the driver's multi-GPU launch shape (torch.distributed.run, one process per
# rank, gloo barrier and max-over-ranks) rehearsed on the one GPU of the box: 2 and 4 ranks all on device 0
# (--devices-same 0), each verifying its own 16,384-set steps; then N=1 for the same box
set -e
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port $((29500 + N)) bench.py --gpus $N --steps 20 --warmup 5 --devices-same 0 \
    > gpurun_out/${TAG}_n$N.json 2> gpurun_out/${TAG}_n$N.err
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/${TAG}_n1.json \
  2> gpurun_out/${TAG}_n1.err
