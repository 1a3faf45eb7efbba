#!/bin/bash
# ab_kstats.sh [ROUNDS]: rocprofv3 kernel statistics of the default build and every
# build/variants/libgsr_*.so, ROUNDS times in alternating order (default 2): per build the
# average duration of the main kernels over ~55 launches each -- steadier than stage events.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=${1:-2}
mkdir -p gpurun_out/abk
K=${AB_KERNELS:-"k_render_bwd1 k_render_fwd k_gaussian_backward k_preprocess k_tiles_scatter"}
shopt -s nullglob
for r in $(seq 1 $R); do
  for so in "" build/variants/libgsr_*.so; do
    name=$(basename "${so:-default}" .so)
    if [ -n "$so" ]; then export GSR_LIBRARY=$PWD/$so; else unset GSR_LIBRARY; fi
    d=gpurun_out/abk/${name}_$r
    rm -rf $d
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --config ${CONFIG:-mt} --steps ${AB_STEPS:-50} --warmup 5 \
      --no-cpu-baseline --no-train --batched-views 1 > $d.log 2>&1 || { echo "$name failed"; tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== $name r$r $(python tools/kstats.py $f | awk -v K="$K" 'BEGIN{split(K,a," ");for(i in a)w[a[i]]=1} {split($1,b,"<"); if (b[1] in w) printf "%s=%s ", b[1], $5}')"
  done
done
