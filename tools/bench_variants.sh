#!/bin/bash
# Bench every build/variants/libgsr_*.so (stage table) after the default build.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
shopt -s nullglob
for so in "" build/variants/libgsr_*.so; do
  name=${so:-default}
  if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
  timeout -k 10 200 python bench.py --stages --no-cpu-baseline --no-train --steps 30 > gpurun_out/bv.json 2> gpurun_out/bv.err || { echo "$name failed"; tail -5 gpurun_out/bv.err; exit 1; }
  echo "== $name $(python -c "import json;d=json.load(open('gpurun_out/bv.json'));print(d['value'], d['ms_per_step'])")"
  grep -v amdgpu.ids gpurun_out/bv.err
done
