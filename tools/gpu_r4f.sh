#!/bin/bash
# list segments: parity subset, then kernel A/B of checkpoint positions
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "list_segments or split_tiles or c1_config or sh3 or rows_binning" > gpurun_out/seg_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/seg_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/seg_pytest.log | head -20; exit $rc; }
bash tools/ab_kstats.sh 2
