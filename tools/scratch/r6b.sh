#!/bin/bash
# round 6 b: full -m gpu suite, host profile at c1 / mt, driver bench command
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v -s -m gpu --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E " $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python tools/host_overhead.py c1 300 > $O/host_c1.txt 2>&1 || exit 1
timeout -k 10 300 python tools/host_overhead.py mt 200 > $O/host_mt.txt 2>&1 || exit 1
HOST_CPROFILE=1 timeout -k 10 300 python tools/host_overhead.py c1 300 > $O/host_c1_cprofile.txt 2>&1 || exit 1
cat $O/host_c1.txt $O/host_mt.txt
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 400 $O/bench.json
timeout -k 10 300 python tools/fetched_instances.py > $O/fetched_instances.json 2> $O/fetched_instances.err || { tail -5 $O/fetched_instances.err; exit 1; }
cat $O/fetched_instances.err
GSR_LIBRARY=build/diag/libgsr_wtrace.so GSR_BWD_WAVES=4 GSR_FWD_WAVES=5 timeout -k 10 300 python tools/wave_trace.py mt $O/wtrace_mt.npz > $O/wtrace_mt.txt 2>&1 || { tail -5 $O/wtrace_mt.txt; exit 1; }
cat $O/wtrace_mt.txt
