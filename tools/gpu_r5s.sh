#!/bin/bash
# GPU tests + kernel A/B (extra-block slot bases, checkpoint registers) + batched forward streams A/B
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_ab.sh r5s 2 && bash tools/ab_batched_env.sh 2 "GSR_MV_FWD_STREAMS=2" "GSR_MV_FWD_STREAMS=3" "GSR_MV_FWD_STREAMS=4" > gpurun_out/r5s/abs.log 2>&1 && cat gpurun_out/r5s/abs.log
