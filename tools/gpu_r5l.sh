#!/bin/bash
# round-5 session: -m gpu suite + kernel A/B (metric scene and C5) + the driver's bench command
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r5l}
bash tools/gpu_ab.sh $T 2 c5 1 && timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --stages > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err && python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['batched']['value'], d['batched']['ratio_to_value'], {k: v['avg_ms'] for k, v in d['stages'].items()})" gpurun_out/$T/bench.json
