#!/bin/bash
# Quick GPU session: the -m gpu suite (or the pytest args given), a short bench with the
# stage table and a rocprofv3 kernel-stats pass.  Stops at the first failing GPU step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --stages --no-cpu-baseline --no-train --steps 100 > gpurun_out/bench.json 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'batched',d['batched']['value'])"
grep -v amdgpu.ids gpurun_out/bench.err
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train --batched-views 1 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
python tools/kstats.py $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
