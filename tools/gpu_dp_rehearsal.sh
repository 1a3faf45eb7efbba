#!/bin/bash
# Two ranks on one GPU over gloo (GSR_DIST_BACKEND=gloo): exercises bench.py's N>1
# path (both exchanges) on the 1-GPU box.  Timings are not meaningful (gloo copies
# through the host, both ranks share the GPU); the 8-GPU RCCL run is the driver's.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for ex in sh allreduce; do
  GSR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 --exchange $ex \
    --batched-views 4 --no-train --config mt > gpurun_out/dp2_$ex.json 2> gpurun_out/dp2_$ex.err \
    || { echo "dp2 $ex failed"; tail -30 gpurun_out/dp2_$ex.err; exit 1; }
  cat gpurun_out/dp2_$ex.json
done
