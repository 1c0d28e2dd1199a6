#!/bin/bash
# Round 4: wave priorities of the two kernels that share the SIMDs after the ACS -- the
# traceback (s_setprio 3 in the product) and the demod (none).
set -o pipefail
O=gpurun_out/r04y; mkdir -p $O
export TMPDIR=/tmp
BA="--steps 12 --warmup 3 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
for r in 1 2; do for v in cur tbp0 tbp1 dmp2 dmp3; do
  L=sdr-j-dab_amd/lib/variants/libdabgpu_$v.so; [ $v = cur ] && L=sdr-j-dab_amd/lib/libdabgpu.so
  DABGPU_LIB=$L timeout -k 10 300 python3 bench.py $BA > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('$v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), round(a['demod'],3), 'acs', round(k['msc_acs'],3), 'tb', round(k['msc_traceback'],3), d['checked_step']['msc_equal_transmitted'])"
done; done
