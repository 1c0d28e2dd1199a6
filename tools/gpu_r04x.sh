#!/bin/bash
# Round 4: frames per step (F) -- the grids' tails and per-run fixed costs against F.
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for f in 24 32 48; do
  timeout -k 10 300 python3 bench.py --frames $f --steps 12 --warmup 3 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0 > $O/f${f}_$r.log 2>&1 || { tail -5 $O/f${f}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/f${f}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']
print('F=$f $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), 'acs', round(k['msc_acs'],3), 'tb', round(k['msc_traceback'],3), d['checked_step']['msc_equal_transmitted'])"
done; done
