#!/bin/bash
# default bench line (with stages) + configs bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/bench
timeout -k 10 400 python bench.py --stages > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err || { tail -20 gpurun_out/bench/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'batched', d['batched']['value'], 'roof', d['roofline']['avg_launch_ms'], d['roofline']['frac'])
print({k: round(v['avg_ms'],4) for k,v in d['stages'].items()})"
