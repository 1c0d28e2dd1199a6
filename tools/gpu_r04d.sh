#!/bin/bash
# Round 4: the double-recurrence NCO (k_demod.hip) -- soft-value error against the round-3
# exact NCO on the same CFO test, the GPU suite, the demod alone under a carrier offset
# (base = round-3 build, tools/build_ref_variant.sh), then the C3 bench interleaved.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
L=$(pwd)/sdr-j-dab_amd/lib
for v in base cur; do
  lib=$L/libdabgpu.so; [ $v != cur ] && lib=$L/variants/libdabgpu_$v.so
  DABGPU_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "demod_nco" -s -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1
  echo "$v rc=$?"; grep -E "worst" $O/t_$v.log
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "suite rc=$?"; grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -8
for v in base cur base cur; do
  lib=$L/libdabgpu.so; [ $v != cur ] && lib=$L/variants/libdabgpu_$v.so
  DABGPU_LIB=$lib timeout -k 10 200 python3 tools/demod_bench.py --phase 1300 --reps 20 > $O/demod_$v.log 2>&1 || { tail -5 $O/demod_$v.log; exit 1; }
  echo "$v: $(grep -E '^(sync_demod|demod) ' $O/demod_$v.log | cut -c1-90 | tr '\n' ' ')"
done
timeout -k 10 600 tools/gpu_ab.sh r04d_ab 2 "base:X=0" "cur:X=0" || exit 1
