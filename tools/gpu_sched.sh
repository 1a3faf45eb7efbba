#!/bin/bash
# per-kernel scheduler strategies (csrc/Makefile SCHED_*): every GPU test on the default build,
# then kernel stats of the default build against build/variants (tools/ab_kstats.sh)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sched_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/sched_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/sched_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sched_smoke.log 2>&1 || { tail -20 gpurun_out/sched_smoke.log; exit 1; }
echo smoke ok
bash tools/ab_kstats.sh 3
