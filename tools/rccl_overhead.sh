#!/bin/bash
# what does an RCCL communicator in the bench process cost the pipeline?
# One GPU, the C3 bench, interleaved:
#   plain     no process group
#   rccl      a one-rank RCCL group whose communicator exists before the rank-local legs
#             (DAB_RCCL_EARLY=1: one all_reduce on the default group), control collectives on
#             the gloo group (this tree's N > 1 path)
#   rcclctl   the same with the control collectives (barriers around the timed region, the
#             max-over-ranks time, the check gathers) on the RCCL group (DAB_CTL_RCCL=1):
#             round 5's first N > 1 path, which measured ~9 % slower (r05_rccl_overhead_ab.txt)
# then a kernel trace (rocprofv3 --kernel-trace --stats) and one PMC pass of k_acs2 for each.
#   tools/rccl_overhead.sh OUT [REPS]
set -o pipefail
O=$1; REPS=${2:-2}
A="--gpus 1 --steps 12 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --delivered-steps 0 --c5-steps 0 --no-c4-fed"
D="DAB_DIST_FORCE=1 DAB_RCCL_EARLY=1 MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1"
C="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY"
port=29580
for r in $(seq 1 $REPS); do
    tools/gpu.sh $O bench plain_$r $A || exit $?
    port=$((port + 1)); env $D MASTER_PORT=$port tools/gpu.sh $O bench rccl_$r $A || exit $?
    port=$((port + 1)); env $D DAB_CTL_RCCL=1 MASTER_PORT=$port tools/gpu.sh $O bench rcclctl_$r $A || exit $?
done
tools/gpu.sh $O stats plain $A --solo-steps 0 &&
env $D MASTER_PORT=29591 tools/gpu.sh $O stats rccl $A --solo-steps 0 &&
env $D DAB_CTL_RCCL=1 MASTER_PORT=29592 tools/gpu.sh $O stats rcclctl $A --solo-steps 0 &&
tools/gpu.sh $O pmc plain "$C" --c5-steps 0 --no-c4-fed &&
env $D MASTER_PORT=29593 tools/gpu.sh $O pmc rccl "$C" --c5-steps 0 --no-c4-fed &&
env $D DAB_CTL_RCCL=1 MASTER_PORT=29594 tools/gpu.sh $O pmc rcclctl "$C" --c5-steps 0 --no-c4-fed
