#!/bin/bash
# Round 4: soft-value error of the anchor + step-factor NCO against the round-3 exact NCO
# (the same new CFO test on both libraries), then the display-feed tests (pipeline + drop-in).
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
L=$(pwd)/sdr-j-dab_amd/lib
for v in base cur; do
  lib=$L/libdabgpu.so; [ $v != cur ] && lib=$L/variants/libdabgpu_$v.so
  DABGPU_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "demod_nco or demod_matches" -s -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1
  echo "$v rc=$?"; grep -E "worst|passed|failed" $O/t_$v.log
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py -k iq_display tests/test_gpu_dropin.py -s -v --timeout 300 --timeout-method thread > $O/t_display.log 2>&1
echo "display rc=$?"; grep -E "PASS|FAIL|Error|error|display feeds|rms" $O/t_display.log | head -20
