#!/bin/bash
# why does an RCCL communicator in the bench process slow the pipeline?
# One GPU, the C3 bench without a process group and with a one-rank RCCL group whose
# communicator exists before the timed steps (DAB_DIST_FORCE=1 DAB_RCCL_EARLY=1):
#   1. the step time of each (bench line)
#   2. a kernel trace of each (rocprofv3 --kernel-trace --stats): RCCL-side kernels, the
#      in-pipeline spans of k_acs2 / k_demod_wg / k_traceback2
#   3. one PMC pass of each (clock, busy cycles, VALU issue of k_acs2 run alone under the
#      profiler's serialisation)
#   tools/rccl_overhead.sh OUT
set -o pipefail
O=$1
A="--gpus 1 --steps 12 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --delivered-steps 0 --c5-steps 0 --no-c4-fed"
D="DAB_DIST_FORCE=1 DAB_RCCL_EARLY=1 MASTER_ADDR=127.0.0.1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1"
C="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY"
tools/gpu.sh $O bench plain $A &&
env $D MASTER_PORT=29581 tools/gpu.sh $O bench rccl $A &&
tools/gpu.sh $O stats plain $A --solo-steps 0 &&
env $D MASTER_PORT=29582 tools/gpu.sh $O stats rccl $A --solo-steps 0 &&
tools/gpu.sh $O pmc plain "$C" --c5-steps 0 --no-c4-fed &&
env $D MASTER_PORT=29583 tools/gpu.sh $O pmc rccl "$C" --c5-steps 0 --no-c4-fed &&
tools/gpu.sh $O bench plain2 $A
