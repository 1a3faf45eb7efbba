set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=80 timeout -k 10 900 tools/opt_sweep.sh "" "split_fwd_bucket=7" "split_fwd_bucket=9" "split_fwd_bucket=6" "split_bwd_depth=640"
