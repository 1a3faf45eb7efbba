#!/bin/bash
# pmc_sq_ab.sh [LIB ...]: one SQ counter pass (instruction mix, wave cycles) per library
# (default build when no argument), summarised per render kernel -> gpurun_out/pmc_ab/<name>.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-train --batched-views 1"
for so in "${@:-default}"; do
  name=$(basename $so .so)
  if [ "$so" = default ]; then unset GSR_LIBRARY; else export GSR_LIBRARY=$PWD/$so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY --kernel-trace -d $OUT/$name -o run --output-format csv -- $B > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  python3 - $OUT/$name <<'PY' | tee $OUT/$name.txt
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        for key in ("k_render_bwd", "k_render_fwd", "k_gaussian_backward"):
            if key in k:
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(sys.argv[1].split("/")[-1], k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(cs.items())}, "(1e6 per dispatch)")
PY
done
