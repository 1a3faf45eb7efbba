set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "depth_sort or c1_config or table_mode or rows_binning" --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?
tail -2 gpurun_out/t3.log
[ $rc -eq 0 ] || exit $rc
GSR_LIBRARY=$PWD/build/trace/libgsr_strace.so timeout -k 10 200 python tools/sort_trace.py > gpurun_out/sort_trace4.txt 2>&1 || { tail -20 gpurun_out/sort_trace4.txt; exit 1; }
grep -A4 '^hist' gpurun_out/sort_trace4.txt | tail -5
timeout -k 10 500 tools/bench_stage_variants.sh depth_sort scan duplicate tile_sort ranges
