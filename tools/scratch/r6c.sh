#!/bin/bash
# round 6 c: host binding in C++ -- tests, host time A/B, bench
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6c; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_ext.py tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_multiview.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -1 $O/pytest_host.log
for cfg in c1 mt; do
  timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}_cpp.txt 2>&1 || exit 1
  GSR_HOST_EXT=0 timeout -k 10 300 python tools/host_overhead.py $cfg 300 > $O/host_${cfg}_ctypes.txt 2>&1 || exit 1
done
HOST_CPROFILE=1 timeout -k 10 300 python tools/host_overhead.py c1 300 > $O/host_c1_cprofile.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/host_*_cpp.txt $O/host_*_ctypes.txt
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
head -c 300 $O/bench.json; echo
timeout -k 10 400 python3 bench.py --config c1 --steps 200 --warmup 20 --no-train --no-cpu-baseline --batched-views 1 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
head -c 300 $O/bench_c1.json; echo
GSR_HOST_EXT=0 timeout -k 10 400 python3 bench.py --config c1 --steps 200 --warmup 20 --no-train --no-cpu-baseline --batched-views 1 > $O/bench_c1_ctypes.json 2> $O/bench_c1_ctypes.err || { tail -20 $O/bench_c1_ctypes.err; exit 1; }
head -c 300 $O/bench_c1_ctypes.json; echo
