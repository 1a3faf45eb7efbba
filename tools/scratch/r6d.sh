#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6d; rm -rf $O; mkdir -p $O
GSR_LIBRARY=build/diag/libgsr_wtrace.so GSR_BWD_WAVES=4 GSR_FWD_WAVES=5 timeout -k 10 300 python tools/wave_trace.py mt $O/wtrace_mt.npz > $O/wtrace_mt.txt 2>&1 || { tail -5 $O/wtrace_mt.txt; exit 1; }
grep "== \|SIMD" $O/wtrace_mt.txt
