#!/bin/bash
# gpu_final.sh TAG: end-of-round numbers beside round_profile.sh -> gpurun_out/TAG/
#   the driver's bench command (N=1), the world-1 RCCL rehearsal of the N>1 path
#   (GSR_DIST_FORCE=1: every step's exchange runs through RCCL), and configs_bench.sh.
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-final}
O=gpurun_out/$TAG
rm -rf $O; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err || { tail -20 $O/driver_cmd.err; exit 1; }
cat $O/driver_cmd.json
GSR_DIST_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 1 --steps 20 --warmup 5 > $O/rccl_world1.json 2> $O/rccl_world1.err || { tail -20 $O/rccl_world1.err; exit 1; }
cat $O/rccl_world1.json
bash tools/configs_bench.sh > $O/configs.txt 2>&1 || { tail -20 $O/configs.txt; exit 1; }
cat $O/configs.txt
