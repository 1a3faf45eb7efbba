#!/bin/bash
# host-route tests on the current binding, then the level-2 chunk / grid variant A/B
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_host_autograd.py tests/test_gpu_host_ext.py tests/test_gpu_api.py > gpurun_out/r6h_pytest.log 2>&1 || { tail -30 gpurun_out/r6h_pytest.log; exit 1; }
tail -1 gpurun_out/r6h_pytest.log
PARITY_K="c1_config or sh3 or rows_binning or background or list_segments" AB_KERNELS="k_tiles_scatter k_tiles_count k_rows_scatter k_rows_count k_render_fwd" bash tools/gpu_abv.sh 2 > gpurun_out/abv_rb.txt 2>&1 || { tail -20 gpurun_out/abv_rb.txt; exit 1; }
grep -E "^parity|^==" gpurun_out/abv_rb.txt
