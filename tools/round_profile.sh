#!/bin/bash
# round_profile.sh TAG: the round's evidence in one GPU session -> gpurun_out/TAG/
#   pytest -m gpu, the default bench line (CPU baseline, train step), rocprofv3 kernel
#   stats of a 30-step bench, and the PMC passes (tools/pmc.sh) summarised.
# Stops at the first failing step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-latest}
O=gpurun_out/$TAG
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
# the driver's bench command, then the same command under the profiler (its kernel statistics are
# the ones the line's roofline avg_launch_ms must agree with)
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stages > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json; grep -v amdgpu.ids $O/bench.err
timeout -k 10 400 python bench.py --stages > $O/bench_200.json 2> $O/bench_200.err || { tail -30 $O/bench_200.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof_bench.log || { tail -20 $O/prof_bench.log; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python tools/kstats.py $O/kernel_stats.csv
for k in k_render_bwd1 k_render_fwd; do python tools/ktrace_phases.py $(find $O/prof -name "*kernel_trace.csv" | head -1) $k; done | tee $O/kernel_phases.txt
bash tools/pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python tools/pmc_summary.py $O/pmc_summary.json | grep -E "^render|^gaussian|^preprocess|^k_tiles|^k_rows"
GSR_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-train > $O/gloo2.json 2> $O/gloo2.err || { tail -20 $O/gloo2.err; exit 1; }
bash tools/configs_bench.sh > $O/configs.txt 2>&1 || { tail -20 $O/configs.txt; exit 1; }
cat $O/configs.txt
# host time per view through the drop-in API (the C++ autograd function, the Python one over the
# C++ binding, and the ctypes route)
for cfg in c1 mt; do
  timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}.txt 2>&1 || exit 1
  GSR_HOST_AUTOGRAD=0 timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}_pyfn.txt 2>&1 || exit 1
  GSR_HOST_EXT=0 timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}_ctypes.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/host_*.txt
# instances the render kernels read (GSR_STATS build) and the per-config roofline from them
if [ -f build/diag/libgsr_stats.so ]; then
  timeout -k 10 300 python tools/fetched_instances.py > $O/fetched_instances.json 2> $O/fetched_instances.err || { tail -5 $O/fetched_instances.err; exit 1; }
  python tools/config_roofline.py gpurun_out/configs $O/fetched_instances.json | tee $O/config_roofline.txt
fi
