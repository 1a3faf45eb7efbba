set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSR_LIBRARY=$PWD/build/trace/libgsr_stats.so timeout -k 10 200 python tools/render_stats.py > gpurun_out/rstats.txt 2>&1 || { tail gpurun_out/rstats.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/rstats.txt
timeout -k 10 500 tools/bench_stage_variants.sh duplicate tile_sort render_fwd render_bwd
