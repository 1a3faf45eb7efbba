set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "split_tiles or c1_config or rows_binning" --timeout 300 --timeout-method thread > gpurun_out/t16.log 2>&1; rc=$?
tail -2 gpurun_out/t16.log
[ $rc -eq 0 ] || exit $rc
STEPS=80 timeout -k 10 900 tools/opt_sweep.sh "" "split4_fwd_bucket=9" "split4_fwd_bucket=10" "split4_fwd_bucket=11" "split4_fwd_bucket=12"
