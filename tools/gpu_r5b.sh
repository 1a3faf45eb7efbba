#!/bin/bash
# Round-5 session b: the precise independent-exp parity test, rocprof A/B of the variant
# builds in build/variants (metric scene, 2 rounds; C5 for the preprocess variant), and the
# driver's bench command.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest tests/test_gpu_exp_budget.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5b/exp.log 2>&1 || { tail -40 gpurun_out/r5b/exp.log; exit 1; }
grep -E "flipped|HIP vs|G vs|unpinned|passed|failed" gpurun_out/r5b/exp.log
bash tools/ab_kstats.sh 2 > gpurun_out/r5b/ab.log 2>&1 || { tail -20 gpurun_out/r5b/ab.log; exit 1; }
cat gpurun_out/r5b/ab.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5b/bench.json 2> gpurun_out/r5b/bench.err || { tail -30 gpurun_out/r5b/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5b/bench.json')); r=d['roofline']; b=d['batched']
print(d['value'], r['avg_launch_ms'], r['avg_launch_ms_timed_region'], r['avg_launch_ms_stage_pass'], r['launches_timed'])
print(b['value'], b['ratio_to_value'], b['overlap'])"
mkdir -p build/variants_c5 && mv build/variants/libgsr_early.so build/variants/libgsr_ckn.so build/variants_c5/ 2>/dev/null
CONFIG=c5 AB_STEPS=12 bash tools/ab_kstats.sh 1 > gpurun_out/r5b/ab_c5.log 2>&1 || { tail -20 gpurun_out/r5b/ab_c5.log; exit 1; }
cat gpurun_out/r5b/ab_c5.log
