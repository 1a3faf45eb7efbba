#!/bin/bash
# profile_batched.sh: kernel stats of bench.py's batched (8 views per step) measurement
# alone (--views-per-gpu 8 times the multi-view step as the main line)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pb -o run -- \
  python bench.py --no-cpu-baseline --no-train --views-per-gpu 8 --batched-views 1 --steps 10 --warmup 3 \
  > gpurun_out/pb.json 2> gpurun_out/pb.err
