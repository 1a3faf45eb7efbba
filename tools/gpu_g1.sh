set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knn.py -x -q -k "depth_sort or c1_config or table_mode or knn or rows_binning" --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
tail -3 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
GSR_LIBRARY=$PWD/build/trace/libgsr_strace.so timeout -k 10 200 python tools/sort_trace.py > gpurun_out/sort_trace2.txt 2>&1 || exit 1
tail -28 gpurun_out/sort_trace2.txt
timeout -k 10 400 tools/bench_stage_variants.sh depth_sort scan duplicate tile_sort render_fwd render_bwd
