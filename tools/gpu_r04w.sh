#!/bin/bash
# Round 4: where the DAB+ superframe decode spends its time -- builds with one part left
# out (timing only: their outputs are wrong): window copy, syndromes, AU CRCs, byte output.
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
export TMPDIR=/tmp
BA="--workload c5 --steps 10 --warmup 3 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0 --solo-steps 3"
for r in 1 2; do for v in cur win syn crc out all; do
  L=sdr-j-dab_amd/lib/variants/libdabgpu_dpx_$v.so; [ $v = cur ] && L=sdr-j-dab_amd/lib/libdabgpu.so
  for sp in 0 1; do
  DABGPU_DP_SPLIT=$sp DABGPU_LIB=$L timeout -k 10 300 python3 bench.py $BA > $O/c5_${v}_${sp}_$r.log 2>&1 || { tail -5 $O/c5_${v}_${sp}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}_${sp}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('$v split=$sp $r', round(d['value']/1e6,2), 'dabplus pipe', round(k['dabplus'],3), 'alone', round(a['dabplus'],3))"
  done
done; done
