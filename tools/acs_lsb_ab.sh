#!/bin/bash
# The ACS with the decision in the metrics' LSB (ACS_LSB=1, the build in lib/: own / partner
# candidates, no subtract) against the lower / upper form with sign-bit decisions
# (ACS_LSB=0), interleaved, solo legs on.  Viterbi + pipeline parity on the new build first.
#   tools/acs_lsb_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
V=$PWD/sdr-j-dab_amd/lib/variants
mkdir -p gpurun_out/$O
timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/$O/tests.log 2>&1 || { tail -30 gpurun_out/$O/tests.log; exit 1; }
tail -2 gpurun_out/$O/tests.log
BENCH_ARGS="--solo-steps 3 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0 --no-c4-fed" \
    bash tools/ab_libs.sh $REPS $V/libdabgpu_lsb.so $V/libdabgpu_nolsb.so | tee gpurun_out/$O/ab.txt
