#!/bin/bash
# parity of the variants, then kernel stats at C5 and the metric scene
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
K=${PARITY_K:-"c1_config or sh3 or list_segments or background or active_degree"}
for so in build/variants/libgsr_*.so; do
  GSR_LIBRARY=$PWD/$so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "$K" > gpurun_out/abv_pytest.log 2>&1; rc=$?
  echo "parity $(basename $so): $(tail -1 gpurun_out/abv_pytest.log)"
  [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/abv_pytest.log | head -10; exit $rc; }
done
CONFIG=c5 AB_STEPS=10 bash tools/ab_kstats.sh 2 || exit 1
bash tools/ab_kstats.sh 2
