#!/bin/bash
# ab_batched_env.sh ROUNDS "ENV=V ..." ...: views/s of the batched mode (8 views per step: per-view
# forwards, one multi-view backward) under each environment setting, ROUNDS times alternating.
set -o pipefail
cd "$(dirname "$0")/.."
R=$1; shift
mkdir -p gpurun_out/abbe
for r in $(seq 1 $R); do
  i=0
  for envs in "$@"; do
    i=$((i + 1))
    d=gpurun_out/abbe/s${i}_$r
    env $envs timeout -k 10 240 python3 bench.py --steps 40 --warmup 8 --views-per-gpu 8 --batched-views 1 \
      --no-cpu-baseline --no-train > $d.json 2> $d.log || { echo "[$envs] failed"; tail -5 $d.log; exit 1; }
    echo "== [$envs] r$r value=$(python3 -c "import json;d=json.load(open('$d.json'));print(d['value'], d['ms_per_step'])")"
  done
done
