#!/bin/bash
# deferred multi-view forward: GPU tests, batched A/B (deferred vs waiting per view), driver bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/ab_batched_env.sh 3 "GSR_MV_DEFERRED=1" "GSR_MV_DEFERRED=0" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stages > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['batched']['value'], d['batched']['ratio_to_value'], d['batched']['overlap']['busy_over_wall'])" $O/bench.json
