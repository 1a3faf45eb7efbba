#!/bin/bash
# opt_sweep.sh "OPTS1" "OPTS2" ...: one short bench per GSR_OPTIONS string (stage table), twice
# over in alternating order so drift between runs shows.  "" = defaults.
# e.g. tools/opt_sweep.sh "" "split_fwd_bucket=10" "split_bwd_depth=512"
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STEPS=${STEPS:-60}
for round in 1 2; do
  for o in "$@"; do
    GSR_OPTIONS="$o" timeout -k 10 200 python bench.py --stages --no-cpu-baseline --no-train --batched-views 1 \
      --steps $STEPS --warmup 10 > gpurun_out/os.json 2> gpurun_out/os.err || { echo "[$o] failed"; tail -5 gpurun_out/os.err; exit 1; }
    v=$(python -c "import json;d=json.load(open('gpurun_out/os.json'));print(d['value'], d['ms_per_step'])")
    st=$(grep -E "^(render_fwd|render_bwd|depth_sort|tile_sort|duplicate|gaussian_bwd) " gpurun_out/os.err | awk '{printf "%s %s  ", $1, $2}')
    echo "[$o] $v | $st"
  done
done
