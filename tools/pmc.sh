#!/bin/bash
# Counter passes (each in its own rocprofv3 run, --kernel-trace only besides --pmc):
#   1: FETCH_SIZE   2: WRITE_SIZE   3: SQ instruction/wait mix
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-train"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
find $OUT -name "*.csv" | head -20
