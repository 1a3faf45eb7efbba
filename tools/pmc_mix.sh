#!/bin/bash
# pmc_mix.sh: instruction mix and LDS/SALU stall counters per kernel (two passes, each its
# own rocprofv3 run) -> gpurun_out/pmc_mix/{a,b}.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mix${CONFIG:+_$CONFIG}
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-train --batched-views 1 ${CONFIG:+--config $CONFIG}"
A="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU"
Bc="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU"
i=0
for set in "$A" "$Bc"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $OUT/p$i -o run --output-format csv -- $B > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, re
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r.get("Kernel_Name", ""))
        if m: acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ("k_render_bwd", "k_render_bwd1", "k_render_fwd", "k_gaussian_backward", "k_tiles_scatter", "k_preprocess", "k_rows_scatter", "k_tiles_count", "k_radix_scatter_grp"):
    if k in acc:
        print(k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(acc[k].items())})
PY
