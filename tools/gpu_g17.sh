set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knn.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t17.log 2>&1; rc=$?
tail -2 gpurun_out/t17.log
[ $rc -eq 0 ] || exit $rc
GSR_LIBRARY=$PWD/build/trace/libgsr_strace.so timeout -k 10 200 python tools/sort_trace.py > gpurun_out/sort_trace6.txt 2>&1 || { tail -20 gpurun_out/sort_trace6.txt; exit 1; }
sed -n '/repetition 2/,$p' gpurun_out/sort_trace6.txt | grep -v XCC
for i in 1 2; do timeout -k 10 500 tools/bench_stage_variants.sh depth_sort render_fwd render_bwd; done
bash tools/configs_bench.sh
