#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
PARITY_K="c1_config or sh3_ragged or background" bash tools/gpu_abv.sh 2 || exit 1
bash tools/opt_sweep.sh "" "split_fwd_bucket=7" "split_fwd_bucket=9"
