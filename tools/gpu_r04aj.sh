#!/bin/bash
# Round 4: same-box A/B -- ACS candidates of the xor-4 / xor-8 steps through the LDS crossbar
# (two ds_swizzle + two adds, variants/libdabgpu_swz48.so) against the product's two plain
# adds + two bank-masked DPP adds.
set -o pipefail
O=gpurun_out/r04aj; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/sdr-j-dab_amd/lib/variants/libdabgpu_swz48.so
DABGPU_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -m gpu -x -v --timeout 300 --timeout-method thread -k "viterbi or profile or c3_full" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for v in prod swz; do
  if [ $v = swz ]; then export DABGPU_LIB=$V; else unset DABGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --delivered-steps 0 > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'acs', round(k['msc_acs'],3), 'alone', round(a['msc_acs'],3), 'demod', round(k['demod'],3), d['checked_step']['msc_equal_transmitted'])"
done; done
