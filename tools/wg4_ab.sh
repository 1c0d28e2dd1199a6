#!/bin/bash
# Demod chunking with 4 resident workgroups per CU assumed (DEMOD_CHUNK_WG_PER_CU=4: C3 splits
# every frame in 2 chunks) against the product's 3 (one chunk per frame), interleaved.
#   tools/wg4_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
V=$PWD/sdr-j-dab_amd/lib/variants
mkdir -p gpurun_out/$O
BENCH_ARGS="--solo-steps 2 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0" \
    bash tools/ab_libs.sh $REPS $V/libdabgpu_r06main.so $V/libdabgpu_r06wg4.so | tee gpurun_out/$O/ab.txt
