#!/bin/bash
# cfgbench.sh [CONFIG ...]: row binning (GSR_ROWS_BINNING=1) vs duplicate + radix tile
# sort (=0) per BASELINE config, views/s and the binning stage times.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "${@:-mt c2 c3 c5}"; do for rb in 1 0; do
 GSR_ROWS_BINNING=$rb timeout -k 10 200 python bench.py --config $cfg --stages --no-cpu-baseline --no-train --steps 50 --warmup 5 --batched-views 1 > gpurun_out/cb.json 2> gpurun_out/cb.err || { tail -5 gpurun_out/cb.err; exit 1; }
 echo "== $cfg rows=$rb $(python -c "import json;d=json.load(open('gpurun_out/cb.json'));print(d['value'], d['ms_per_step'])")"
 grep -E "duplicate|tile_sort|ranges" gpurun_out/cb.err
done; done
