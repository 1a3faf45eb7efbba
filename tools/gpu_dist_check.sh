#!/bin/bash
# the multi-GPU path on one box: dist tests (gloo x2, RCCL world 1 torch and native), then the
# bench's RCCL world-1 rehearsal (native exchange, teardown included)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_c4.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/dist_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/dist_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|failed" gpurun_out/dist_pytest.log | head -20; exit $rc; }
bash tools/gpu_rccl_w1.sh
