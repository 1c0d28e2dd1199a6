#!/bin/bash
# Round 6: demod variants against the round-5 kernel: one PMC pass of each library (VALU /
# LDS instructions, LDS bank conflicts, clock) over the C3 bench step, then interleaved bench
# runs (tools/ab_libs.sh).
#   tools/demod_ab.sh OUT REPS LIB...
set -o pipefail
O=$1; REPS=$2; shift 2
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for L in "$@"; do
    n=$(basename "$L" .so)
    DABGPU_LIB=$L tools/gpu.sh $O pmc $n "$C" --c5-steps 0 --no-c4-fed || exit $?
done
BENCH_ARGS="--solo-steps 2 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0" bash tools/ab_libs.sh $REPS "$@" | tee gpurun_out/$O/ab.txt
