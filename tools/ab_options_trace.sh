#!/bin/bash
# ab_options_trace.sh CONFIG "OPTS_A" ["OPTS_B" ...]: rocprofv3 kernel statistics of a 100-step bench
# at CONFIG under each GSR_OPTIONS setting (runtime options, one build) -> gpurun_out/optrace/
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
cfg=$1; shift; O=gpurun_out/optrace; mkdir -p $O
i=0
for opt in "$@"; do
  i=$((i + 1))
  GSR_OPTIONS="$opt" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$i -o kt --output-format csv -- \
    python3 bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-train --batched-views 1 \
    > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  echo "== $cfg [$opt] views/s $(python3 -c "import json;print(json.load(open('$O/b$i.json'))['value'])")"
  python tools/kstats.py $(find $O/p$i -name "*kernel_stats.csv" | head -1) | grep -E "k_render|k_gaussian_backward |k_preprocess"
  rm -rf $O/p$i
done
