#!/bin/bash
# The traceback's register ring 3 deep (the product: 340 VGPRs, one 123-VGPR demod wave
# fits beside a traceback wave on a SIMD) against 2 (255 VGPRs: two demod waves fit) and 1
# (162), interleaved, solo legs on.  Parity tests of the Viterbi on the ring-2 build first.
#   tools/tb_ring_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
V=$PWD/sdr-j-dab_amd/lib/variants
mkdir -p gpurun_out/$O
DABGPU_LIB=$V/libdabgpu_ring2.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -x -q -m gpu \
    -k "viterbi or pipeline or c3 or packed" --timeout 120 --timeout-method thread > gpurun_out/$O/tests.log 2>&1 || { tail -30 gpurun_out/$O/tests.log; exit 1; }
tail -2 gpurun_out/$O/tests.log
BENCH_ARGS="--solo-steps 3 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0 --no-c4-fed" \
    bash tools/ab_libs.sh $REPS $V/libdabgpu_ring3.so $V/libdabgpu_ring2.so $V/libdabgpu_ring1.so | tee gpurun_out/$O/ab.txt
