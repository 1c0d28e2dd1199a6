#!/bin/bash
# Round 4: the demod without the NCO factor tables in LDS (34.8 KB per workgroup, was 40 KB;
# variant ncl = the previous commit) and the traceback's register ring depth (ring1/ring2 =
# TB_RING_DEPTH 1/2, the product 3), in the C3 pipeline; drop-in tests first.
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "dropin or gui or demod" -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo "tests rc=$?"; grep -E "FAILED|passed|failed" $O/t.log | tail -4
timeout -k 10 900 tools/gpu_ab.sh r04e_ab 2 "ncl:X=0" "cur:X=0" "ring1:X=0" "ring2:X=0" || exit 1
