set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSR_LIBRARY=$PWD/build/trace/libgsr_strace.so timeout -k 10 200 python tools/sort_trace.py > gpurun_out/sort_trace3.txt 2>&1 || { tail -20 gpurun_out/sort_trace3.txt; exit 1; }
timeout -k 10 400 tools/bench_stage_variants.sh depth_sort scan duplicate tile_sort ranges
