set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for so in "" build/variants/libgsr_*.so; do
  if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
  timeout -k 10 200 python bench.py --config c1 --steps 100 --warmup 10 --no-cpu-baseline --no-train --batched-views 1 --stages > gpurun_out/c1b.json 2> gpurun_out/c1b.err || { echo "${so} failed"; tail -3 gpurun_out/c1b.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/c1b.json'));print('${so:-default}', d['value'], d['step_ms']['median'], ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['stages'].items()))"
done
