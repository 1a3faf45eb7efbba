#!/bin/bash
# bench_stage_variants.sh [STAGE ...]: value and per-stage ms (default: depth_sort, tile_sort,
# gaussian_bwd) of the default build and every build/variants/libgsr_*.so (single view, no CPU leg)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
stages=${*:-depth_sort tile_sort gaussian_bwd}
shopt -s nullglob
for so in "" build/variants/libgsr_*.so; do
  name=${so:-default}
  if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train --batched-views 1 --steps 100 --warmup 8 \
    > gpurun_out/bs.json 2> gpurun_out/bs.err || { echo "$name failed"; tail -5 gpurun_out/bs.err; exit 1; }
  echo "== $name $(python -c "
import json,sys;d=json.load(open('gpurun_out/bs.json'))
print(d['value'], ' '.join('%s=%.4f' % (s, d['stages'].get(s, {}).get('avg_ms', 0.0)) for s in sys.argv[1:]))" $stages)"
done
