#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -25 gpurun_out/pytest_gpu.log
# A crash, abort or time limit ends the session; an ordinary test failure does not.
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py --stages > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; cat gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json gpurun_out/bench.err
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_bench.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
