#!/bin/bash
# Round 4: same-box A/B -- the next run's front end waiting for run r-1's ACS (the ring's
# last reader, variants/libdabgpu_fafter.so) instead of run r-1's whole back end (product).
set -o pipefail
O=gpurun_out/r04ah; mkdir -p $O
export TMPDIR=/tmp
V=$PWD/sdr-j-dab_amd/lib/variants/libdabgpu_fafter.so
DABGPU_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c3_full or c5_full or dropout or background or lockstep or packed or every_profile" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for v in prod after; do
  if [ $v = after ]; then export DABGPU_LIB=$V; else unset DABGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), 'acs', round(k['msc_acs'],3), 'tb', round(k['msc_traceback'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), d['checked_step']['msc_equal_transmitted'])"
done; done
for v in prod after; do
  if [ $v = after ]; then export DABGPU_LIB=$V; else unset DABGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 > $O/c5_${v}.log 2>&1 || { tail -5 $O/c5_${v}.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}.log') if l.startswith('{')][-1])
print('c5 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2))"
done
