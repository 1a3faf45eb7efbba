#!/bin/bash
# ab_env.sh ROUNDS "ENV=V ..." "ENV=V ..." ...: rocprofv3 kernel statistics of the default build
# under each environment setting (e.g. GSR_TILE_SORT=0 vs 1), ROUNDS times in alternating order,
# metric scene unless CONFIG is set.  Prints per setting the average duration of the main kernels
# and the step's binning-chain sum.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$1; shift
mkdir -p gpurun_out/abe
for r in $(seq 1 $R); do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    d=gpurun_out/abe/s${i}_$r
    rm -rf $d
    env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --config ${CONFIG:-mt} \
      --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline --no-train --batched-views 1 > $d.json 2> $d.log || { echo "[$envs] failed"; tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== [$envs] r$r value=$(python3 -c "import json;print(json.load(open('$d.json'))['value'])")"
    python3 tools/kstats.py $f --per-step k_preprocess | head -24
  done
done
