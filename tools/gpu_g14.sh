set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_api.py -x -q --timeout 400 --timeout-method thread > gpurun_out/t14.log 2>&1; rc=$?
tail -2 gpurun_out/t14.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 500 tools/bench_stage_variants.sh duplicate tile_sort render_fwd render_bwd; done
