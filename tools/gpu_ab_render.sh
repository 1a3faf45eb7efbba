#!/bin/bash
# A/B of render variants: parity subset on the default build, then every build/variants/*.so
# (render stages), twice.  Usage: tools/gpu_ab_render.sh [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q -m gpu --timeout 200 --timeout-method thread ${1:+-k "$1"} > gpurun_out/ab_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/ab_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 600 tools/bench_stage_variants.sh render_fwd render_bwd gaussian_bwd || exit 1; done
