#!/bin/bash
# A/B of runtime options at C1 and C2 (no rebuild): default vs bwd_ckpt 64 / 128
set -o pipefail
cd "$(dirname "$0")/.." 2>/dev/null || true
O=gpurun_out/c1ab; mkdir -p $O
for r in 1 2; do
for opt in "" "bwd_ckpt=64" "bwd_ckpt=128"; do
  for cfg in c1 c2; do
    GSR_OPTIONS="$opt" timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 10 --no-cpu-baseline --no-train --batched-views 1 --stages > $O/$cfg.json 2> $O/$cfg.err || { tail -5 $O/$cfg.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$cfg.json'));print('r$r', '$cfg', '[$opt]', 'views/s', d['value'], 'median', d['step_ms']['median'], ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['stages'].items() if k.startswith('render')))"
  done
done
done
