#!/bin/bash
# One GPU session: the -m gpu suite, smoke, the 2-rank gloo rehearsal of bench.py's own launcher,
# and the driver's bench command.  Usage: tools/gpu_session.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=${1:-r5}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
GSR_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $O/gloo2.json 2> $O/gloo2.err \
  || { tail -30 $O/gloo2.err; exit 1; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
  || { tail -30 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("gloo2", "bench"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    c = d["config"]
    print(f, d["value"], d["ms_per_step"], c.get("world_size"), c.get("dist_backend"), c.get("launcher"),
          (d.get("batched") or {}).get("value"), (d.get("roofline") or {}).get("avg_launch_ms"))
PY
