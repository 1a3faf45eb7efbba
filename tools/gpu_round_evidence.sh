#!/bin/bash
# gpu_round_evidence.sh TAG: the round's evidence on the committed sources -- GPU tests, bench line, kernel
# stats, PMC passes (round_profile.sh), the configs bench and the RCCL world-1 rehearsal -> gpurun_out/TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/round_profile.sh ${1:-round4_c} || exit 1
bash tools/configs_bench.sh c1 c2 mt c3 c5 > gpurun_out/${1:-round4_c}/configs.txt 2>&1 || { tail -5 gpurun_out/${1:-round4_c}/configs.txt; exit 1; }
cat gpurun_out/${1:-round4_c}/configs.txt
bash tools/gpu_rccl_w1.sh || exit 1
