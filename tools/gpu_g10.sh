set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 500 tools/bench_stage_variants.sh preprocess depth_sort scan duplicate tile_sort ranges render_fwd render_bwd; done
