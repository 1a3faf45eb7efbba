#!/bin/bash
# bench line, then preprocess occupancy A/B at C5 and mt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_bench.sh || exit 1
CONFIG=c5 AB_STEPS=10 bash tools/ab_kstats.sh 2 || exit 1
bash tools/ab_kstats.sh 1
