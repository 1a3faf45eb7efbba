#!/bin/bash
# variant A/B with parity: a parity subset on every build/variants/libgsr_*.so (GSR_LIBRARY), then
# rocprofv3 kernel stats of the default build and the variants (tools/ab_kstats.sh)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${PARITY_K:-"c1_config or sh3 or list_segments or background or active_degree"}
for so in build/variants/libgsr_*.so; do
  GSR_LIBRARY=$PWD/$so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "$K" > gpurun_out/abv_pytest.log 2>&1; rc=$?
  echo "parity $(basename $so): $(tail -1 gpurun_out/abv_pytest.log)"
  [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/abv_pytest.log | head -10; exit $rc; }
done
bash tools/ab_kstats.sh ${1:-2}
