#!/bin/bash
# GPU session: hardware exp2 characterisation + parity budgets of the default and fast-exp builds.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PROBE" ]; then
  timeout -k 10 120 tools/bin/exp_probe -8.125 > gpurun_out/exp_probe.txt 2>&1 || exit $?
  cat gpurun_out/exp_probe.txt
fi
timeout -k 10 400 python -u tools/parity_budget.py ${CASES:-c1 sh3 bgmod large c2 mt} > gpurun_out/budget_default.jsonl 2> gpurun_out/budget_default.err || { tail gpurun_out/budget_default.err; exit 1; }
GSR_LIBRARY=$PWD/build/variants/libgsr_fastexp.so timeout -k 10 400 python -u tools/parity_budget.py ${CASES:-c1 sh3 bgmod large c2 mt} > gpurun_out/budget_fastexp.jsonl 2> gpurun_out/budget_fastexp.err || { tail gpurun_out/budget_fastexp.err; exit 1; }
echo done
