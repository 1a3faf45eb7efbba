#!/bin/bash
# full GPU test suite, then kernel A/B against build/variants
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash tools/ab_kstats.sh ${1:-2}
