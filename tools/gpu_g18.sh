set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_knn.py tests/test_gpu_c4.py -x -q --timeout 400 --timeout-method thread > gpurun_out/t18.log 2>&1; rc=$?
tail -2 gpurun_out/t18.log
[ $rc -eq 0 ] || exit $rc
for cfg in c3 c5 mt; do
for so in "" build/variants/libgsr_head.so; do
  if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
  timeout -k 10 300 python bench.py --config $cfg --steps 60 --warmup 10 --no-cpu-baseline --no-train --batched-views 1 --stages > gpurun_out/cf.json 2> gpurun_out/cf.err || { tail -3 gpurun_out/cf.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/cf.json'));print('$cfg ${so:-default}', d['value'], d['step_ms']['median'], ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['stages'].items()))"
done; done
