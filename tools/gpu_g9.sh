set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/t9.log 2>&1; rc=$?
tail -2 gpurun_out/t9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 tools/bench_stage_variants.sh depth_sort scan duplicate tile_sort ranges render_fwd render_bwd
timeout -k 10 500 tools/bench_stage_variants.sh depth_sort scan duplicate tile_sort ranges render_fwd render_bwd
