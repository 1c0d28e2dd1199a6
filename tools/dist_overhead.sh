#!/bin/bash
# Does the process group in the bench process change the pipeline's step time?  One GPU:
# the same bench command without a process group and with a one-rank RCCL default group
# (DAB_DIST_FORCE=1; its control collectives go through the gloo group), then the C4 leg's
# RCCL transfers after the rank-local legs (u8 and s16 wire formats).
#   tools/dist_overhead.sh OUT
set -o pipefail
O=$1
A="--gpus 1 --steps 12 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --delivered-steps 0"
D="DAB_DIST_FORCE=1 MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1"
tools/gpu.sh $O bench plain $A --no-c4-fed &&
env $D MASTER_PORT=29571 tools/gpu.sh $O bench rccl $A --no-c4-fed &&
env $D MASTER_PORT=29572 tools/gpu.sh $O bench rccl_c4 $A --fed-steps 4 &&
env $D MASTER_PORT=29573 tools/gpu.sh $O bench rccl_c4s16 $A --fed-steps 3 --fed-format s16 &&
tools/gpu.sh $O bench plain2 $A --no-c4-fed
