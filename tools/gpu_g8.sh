set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-train --batched-views 1 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
python tools/timeline.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) > gpurun_out/timeline.txt
cat gpurun_out/timeline.txt
python tools/kstats.py $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
