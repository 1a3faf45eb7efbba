#!/bin/bash
# RCCL world-size-1 rehearsal of the N-GPU exchange (GSR_DIST_FORCE=1: a process group at
# world size 1, so the collectives, the SH rebuild and their overlap with the next step run
# as the N-GPU bench issues them), beside the no-exchange bench: value per mode.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/rccl
STEPS=${STEPS:-100}
export GSR_HOST_PROFILE=1
timeout -k 10 300 python bench.py --steps $STEPS --warmup 10 --no-cpu-baseline --no-train --batched-views 1 \
  > gpurun_out/rccl/none.json 2> gpurun_out/rccl/none.err || { tail -20 gpurun_out/rccl/none.err; exit 1; }
for ex in sh allreduce; do
  GSR_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --steps $STEPS --warmup 10 --exchange $ex \
    --no-cpu-baseline --no-train --batched-views 1 > gpurun_out/rccl/$ex.json 2> gpurun_out/rccl/$ex.err \
    || { echo "rccl $ex failed"; tail -30 gpurun_out/rccl/$ex.err; exit 1; }
done
python - <<'PY'
import json
for m in ("none", "sh", "allreduce"):
    d = json.load(open(f"gpurun_out/rccl/{m}.json"))
    ex = d.get("exchange") or {}
    print(m, d["value"], d["ms_per_step"], d["config"].get("dist_backend"), ex.get("chosen"), d.get("host_us_per_step"),
          json.dumps(ex.get("model_us")))
PY
