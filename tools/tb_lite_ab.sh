#!/bin/bash
# The lean traceback (TB_LITE) against the product's: parity of the variant on the pipeline
# tests, then interleaved bench runs.   tools/tb_lite_ab.sh OUT REPS
# (the variant: git apply tools/tb_lite.patch && tools/build_variant.sh r06tblite -DTB_LITE=1;
#  the base: lib/variants/libdabgpu_r06main.so, a copy of the product's library)
set -o pipefail
O=$1; REPS=${2:-3}
V=$PWD/sdr-j-dab_amd/lib/variants
mkdir -p gpurun_out/$O
DABGPU_LIB=$V/libdabgpu_r06tblite.so tools/gpu.sh $O tests tests/test_gpu_pipeline_oracle.py \
    -k "c3_full or packed or bits_match or dropout or c5_full" || exit $?
BENCH_ARGS="--solo-steps 2 --delivered-steps 0 --sync-loss-steps 0 --c5-steps 0" \
    bash tools/ab_libs.sh $REPS $V/libdabgpu_r06main.so $V/libdabgpu_r06tblite.so | tee gpurun_out/$O/ab.txt
