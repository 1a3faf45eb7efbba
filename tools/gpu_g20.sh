set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSR_LIBRARY=$PWD/build/variants/libgsr_big.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "depth_sort or c1_config or large_gaussians" --timeout 300 --timeout-method thread > gpurun_out/t20.log 2>&1; rc=$?
tail -2 gpurun_out/t20.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 500 tools/bench_stage_variants.sh depth_sort; done
