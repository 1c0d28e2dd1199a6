#!/bin/bash
# Round 3 (third session): traceback ring loads issued by inline asm (counted waits), checked
# and timed against the previous build: GPU tests on the product library, the traceback alone
# (Viterbi operator under rocprofv3), then the C3 bench interleaved base / product.
# Variants: base = tools/build_variant.sh base "" on the product source; asmld/asmld4 = the same
# on the source with tools/tb_asm_ring.patch applied (asmld4: TB_RING set to 4); the record is
# profiles/r03d_tb_asm_ab.txt.
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 tools/gpu_tb.sh base asmld agst agst4 || exit 1
timeout -k 10 600 tools/gpu_ab.sh r03d_ab 3 "base:X=0" "asmld:X=0" "cur:X=0" "agst4:X=0" || exit 1
