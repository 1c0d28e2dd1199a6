#!/bin/bash
# The soft bits' fast path with r1 from two products and two fmas (DEMOD_R1_FMA=1, the build in lib/)
# against the reference's four-rounding r1 (DEMOD_R1_FMA=0), interleaved, solo legs on; all -m gpu tests first.
#   tools/r1fma_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
V=$PWD/sdr-j-dab_amd/lib/variants
mkdir -p gpurun_out/$O
timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/$O/tests.log 2>&1 || { tail -30 gpurun_out/$O/tests.log; exit 1; }
tail -2 gpurun_out/$O/tests.log
BENCH_ARGS="--solo-steps 3 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0 --no-c4-fed" \
    bash tools/ab_libs.sh $REPS $V/libdabgpu_r1fma.so $V/libdabgpu_r1exact.so | tee gpurun_out/$O/ab.txt
