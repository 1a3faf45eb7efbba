#!/bin/bash
# gpu_ab.sh: GPU tests, then the default build against build/variants/libgsr_*.so twice
# (render and binning stages), then a kernel-trace timeline of the default build.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash tools/bench_stage_variants.sh ${AB_STAGES:-render_bwd render_fwd depth_sort} || exit 1
bash tools/bench_stage_variants.sh ${AB_STAGES:-render_bwd render_fwd depth_sort} || exit 1
rm -rf gpurun_out/ab_prof
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab_prof -o kt --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train --batched-views 1 > gpurun_out/ab_prof.log 2>&1 || { tail -20 gpurun_out/ab_prof.log; exit 1; }
python tools/timeline.py "$(find gpurun_out/ab_prof -name "*kernel_trace.csv" -print -quit)" > gpurun_out/ab_timeline.txt && sed -n 1,8p gpurun_out/ab_timeline.txt
