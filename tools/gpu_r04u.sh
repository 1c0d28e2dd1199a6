#!/bin/bash
# Round 4: inverse depuncturing tables as tile-relative bytes (q mod 240, u8 instead of
# u16: one cache line per wave-load instead of two, no offset arithmetic in the scatter).
# Whole GPU suite, then C3 and C5 interleaved against HEAD before the change (prev).
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
BA="--steps 20 --warmup 5 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
for r in 1 2; do for v in cur prev; do
  L=sdr-j-dab_amd/lib/libdabgpu.so; [ $v = prev ] && L=sdr-j-dab_amd/lib/variants/libdabgpu_prev.so
  DABGPU_LIB=$L timeout -k 10 300 python3 bench.py $BA > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), round(a['demod'],3), 'acs', round(k['msc_acs'],3), round(a['msc_acs'],3), 'tb', round(k['msc_traceback'],3), round(a['msc_traceback'],3), 'ok', d['checked_step']['msc_equal_transmitted'])"
done; done
for v in cur prev; do
  L=sdr-j-dab_amd/lib/libdabgpu.so; [ $v = prev ] && L=sdr-j-dab_amd/lib/variants/libdabgpu_prev.so
  DABGPU_LIB=$L timeout -k 10 300 python3 bench.py --workload c5 $BA > $O/c5_${v}.log 2>&1 || { tail -5 $O/c5_${v}.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']
print('c5 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), 'acs', round(k['msc_acs'],3), d['dabplus_last_step'])"
done
