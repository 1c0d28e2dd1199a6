#!/bin/bash
# Round 4: same-box A/B of the DAB+ layer's stream -- product build (layer on a stream of its
# own) against the build with the layer on the run's back-end stream (variants/libdabgpu_base.so).
set -o pipefail
O=gpurun_out/r04af; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for v in base own; do
  if [ $v = base ]; then export DABGPU_LIB=$PWD/sdr-j-dab_amd/lib/variants/libdabgpu_base.so; else unset DABGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --sync-loss-steps 0 > $O/c5_${v}_$r.log 2>&1 || { tail -5 $O/c5_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}_$r.log') if l.startswith('{')][-1]); x=d['delivered']; k=d['kernel_ms_per_launch']
print('c5 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), 'acs', round(k['msc_acs'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3))"
done; done
