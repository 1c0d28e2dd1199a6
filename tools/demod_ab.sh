#!/bin/bash
# Round 6: the demod's 6-slot FFT tail against the round-5 kernel (lib/variants/libdabgpu_r06base.so,
# built from the previous commit): one PMC pass of each (VALU / LDS instructions, LDS bank
# conflicts, clock) over the C3 bench step, then interleaved bench runs (tools/ab_libs.sh).
#   tools/demod_ab.sh OUT BASE_LIB NEW_LIB REPS
set -o pipefail
O=$1; BASE=$2; NEW=$3; REPS=${4:-3}
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
DABGPU_LIB=$BASE tools/gpu.sh $O pmc base "$C" --c5-steps 0 --no-c4-fed &&
DABGPU_LIB=$NEW tools/gpu.sh $O pmc new "$C" --c5-steps 0 --no-c4-fed &&
BENCH_ARGS="--solo-steps 2 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0" bash tools/ab_libs.sh $REPS $BASE $NEW | tee gpurun_out/$O/ab.txt
