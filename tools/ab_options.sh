#!/bin/bash
# ab_options.sh "opt=v,..." "opt=v,..." ...: alternating bench runs (metric scene) of option sets
# (GSR_OPTIONS, applied at import), two rounds; prints views/s and the render stages per run.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/ab_options; mkdir -p $O
CFG=${AB_CONFIG:-mt}
for r in 1 2; do
  for v in "$@"; do
    tag=$(echo "$v" | tr ',=' '__')
    GSR_OPTIONS="$v" timeout -k 10 200 python3 bench.py --config $CFG --steps 100 --warmup 10 --no-train --no-cpu-baseline --batched-views 1 > $O/$tag.r$r.json 2> $O/$tag.r$r.err || { tail -5 $O/$tag.r$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$tag.r$r.json'));s=d['stages'];print('r$r', '%-28s'%'$v', d['value'], 'med', d['step_ms']['median'], ' '.join('%s=%.4f'%(k,s[k]['avg_ms']) for k in ('render_fwd','render_bwd','tile_sort') if k in s))"
  done
done
