#!/bin/bash
# rocprof A/B only: default build vs build/variants/libgsr_*.so at the metric scene.  Usage: tools/gpu_abonly.sh TAG [ROUNDS]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-abonly}
mkdir -p $O
bash tools/ab_kstats.sh ${2:-2} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
