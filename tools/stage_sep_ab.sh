#!/bin/bash
# The demod's soft-bit stage in LDS of its own (DEMOD_STAGE_SEP=1, the build in lib/:
# 4 workgroup barriers per symbol) against the stage in the FFT exchange buffer
# (DEMOD_STAGE_SEP=0: 6 barriers), interleaved, solo legs on.
#   tools/stage_sep_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
V=$PWD/sdr-j-dab_amd/lib/variants
mkdir -p gpurun_out/$O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -x -q -m gpu \
    --timeout 120 --timeout-method thread > gpurun_out/$O/tests.log 2>&1 || { tail -30 gpurun_out/$O/tests.log; exit 1; }
tail -2 gpurun_out/$O/tests.log
BENCH_ARGS="--solo-steps 3 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0 --no-c4-fed" \
    bash tools/ab_libs.sh $REPS $V/libdabgpu_sep.so $V/libdabgpu_nosep.so | tee gpurun_out/$O/ab.txt
