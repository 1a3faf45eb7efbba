#!/bin/bash
# Kernel trace of the batched mode (8 views per step: per-view forwards on two streams, one
# multi-view backward) and of the single-view mode, for tools/timeline.py / kstats.py.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-bprof}
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/b8 -o kt --output-format csv -- python3 bench.py --steps 40 --warmup 8 \
  --views-per-gpu 8 --batched-views 1 --no-cpu-baseline --no-train > $O/b8.json 2> $O/b8.log || { tail -20 $O/b8.log; exit 1; }
python3 tools/kstats.py $(find $O/b8 -name "*kernel_stats.csv" | head -1) --per-step k_gaussian_backward_mv | head -30
python3 -c "import json;d=json.load(open('$O/b8.json'));print('batched-mode value', d['value'], d['ms_per_step'])"
