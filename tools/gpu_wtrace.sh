#!/bin/bash
# wave timelines of the render kernels (GSR_WAVE_TRACE build) at the metric scene
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wtrace
GSR_LIBRARY=build/diag/libgsr_wtrace.so timeout -k 10 300 python tools/wave_trace.py ${1:-mt} gpurun_out/wtrace/${1:-mt}.npz 2>&1 | grep -v amdgpu.ids
