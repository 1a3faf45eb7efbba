#!/bin/bash
# GPU session: the -m gpu suite, then a rocprof A/B of the default build against every
# build/variants/libgsr_*.so (tools/ab_kstats.sh; metric scene, ROUNDS rounds; optionally C5).
# Usage: tools/gpu_ab.sh TAG [ROUNDS] [c5 [C5_ROUNDS]]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=${1:-ab}; R=${2:-2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/ab_kstats.sh $R > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
if [ "$3" = "c5" ]; then
  CONFIG=c5 AB_STEPS=12 bash tools/ab_kstats.sh ${4:-1} > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; exit 1; }
  cat $O/ab_c5.log
fi
