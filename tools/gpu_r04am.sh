#!/bin/bash
# Round 4: more same-box passes of the stage-layout A/B (20 steps each, alternating).
set -o pipefail
O=gpurun_out/r04am; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/sdr-j-dab_amd/lib/variants/libdabgpu_base.so
for r in 1 2 3; do for v in new base; do
  if [ $v = base ]; then export DABGPU_LIB=$V; else unset DABGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-loss-steps 0 --delivered-steps 0 > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod alone', round(a['demod'],3), 'acs', round(k['msc_acs'],3), 'acs alone', round(a['msc_acs'],3))"
done; done
