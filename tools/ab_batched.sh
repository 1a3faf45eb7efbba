#!/bin/bash
# ab_batched.sh [ROUNDS]: the batched mode (8 views per step, one multi-view backward) of the default
# build and every build/variants/libgsr_*.so, ROUNDS times in alternating order: views/s and the
# multi-view kernel's rocprofv3 average.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${1:-2}
mkdir -p gpurun_out/abb
shopt -s nullglob
for r in $(seq 1 $R); do
  for so in "" build/variants/libgsr_*.so; do
    name=$(basename "${so:-default}" .so)
    if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
    d=gpurun_out/abb/${name}_$r
    rm -rf $d
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --steps 40 --warmup 8 \
      --views-per-gpu 8 --batched-views 1 --no-cpu-baseline --no-train > $d.json 2> $d.log || { echo "$name failed"; tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== $name r$r value $(python3 -c "import json,sys;print(json.load(open(sys.argv[1]))['value'])" $d.json) $(python tools/kstats.py $f | grep -E "k_gaussian_backward_mv|k_sh_dsh" | tr -s " " | cut -d" " -f1,5 | tr "\n" " ")"
  done
done
