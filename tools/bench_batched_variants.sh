#!/bin/bash
# bench_batched_variants.sh: the batched (8 views per step) value for the default build and
# every build/variants/libgsr_*.so
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
shopt -s nullglob
for so in "" build/variants/libgsr_*.so; do
  name=${so:-default}
  if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train --steps 80 --warmup 8 > gpurun_out/bb.json 2> gpurun_out/bb.err || { echo "$name failed"; tail -5 gpurun_out/bb.err; exit 1; }
  echo "== $name $(python -c "import json;d=json.load(open('gpurun_out/bb.json'));print('single', d['value'], 'batched', d['batched']['value'], d['batched']['ms_per_step'])")"
done
