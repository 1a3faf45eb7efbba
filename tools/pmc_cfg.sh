#!/bin/bash
# pmc_cfg.sh CONFIG [KERNEL_REGEX]: HBM bytes (FETCH_SIZE, WRITE_SIZE passes) and the SQ mix of one
# bench config's kernels -> gpurun_out/pmc_CONFIG/ (each counter group in its own rocprofv3 run).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
C=${1:-c5}
OUT=gpurun_out/pmc_$C
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-train --batched-views 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
python tools/kstats.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) | head -12
