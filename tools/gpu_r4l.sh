#!/bin/bash
# native RCCL exchange: dist tests, RCCL world-1 rehearsal (native and torch paths)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/dist_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/dist_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|failed" gpurun_out/dist_pytest.log | head -20; exit $rc; }
bash tools/gpu_rccl_w1.sh || exit 1
mkdir -p gpurun_out/rccl_torch
for ex in sh allreduce; do
  GSR_NATIVE_DP=0 GSR_DIST_FORCE=1 GSR_HOST_PROFILE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29523 bench.py --steps 100 --warmup 10 --exchange $ex \
    --no-cpu-baseline --no-train --batched-views 1 > gpurun_out/rccl_torch/$ex.json 2> gpurun_out/rccl_torch/$ex.err \
    || { echo "torch $ex failed"; tail -20 gpurun_out/rccl_torch/$ex.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rccl_torch/$ex.json'));print('torch', '$ex', d['value'], d['ms_per_step'], d['exchange']['issued_by'], d.get('host_us_per_step'))"
done
