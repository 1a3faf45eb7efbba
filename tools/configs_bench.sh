#!/bin/bash
# configs_bench.sh [CONFIG ...]: one bench line per BASELINE config on one GPU
# (gsr_tools.scene.CONFIGS; default c1 c2 mt c3 c5) -> gpurun_out/configs/<cfg>.json
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/configs
for cfg in ${@:-c1 c2 mt c3 c5}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-train --batched-views 1 --stages \
    > gpurun_out/configs/$cfg.json 2> gpurun_out/configs/$cfg.err || { tail -5 gpurun_out/configs/$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/configs/$cfg.json'));c=d['config'];r=d['roofline'];print('$cfg', c['P'], c['width'], c['height'], 'I', c['num_rendered'], 'views/s', d['value'], 'ms', d['ms_per_step'], 'median', d['step_ms']['median'], 'p90', d['step_ms']['p90'], 'view_frac', r['whole_view_frac']); print('   ', ' '.join('%s=%.4f' % (k, v['avg_ms']) for k, v in d['stages'].items()))"
done
