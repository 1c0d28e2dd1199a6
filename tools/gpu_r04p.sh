#!/bin/bash
# Round 4: dabgpu_pipe_fetch through k_to_host (a few waves writing the mapped pinned buffer)
# vs the runtime's copy (DABGPU_D2H_WGS=0); grid sizes 4 / 8 / 32 workgroups.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
export TMPDIR=/tmp
BA="--steps 10 --warmup 3 --no-cpu-baseline --solo-steps 0 --sync-loss-steps 0 --delivered-steps 10"
for r in 1 2; do for w in 2 4 8 16; do
  DABGPU_D2H_WGS=$w timeout -k 10 300 python3 bench.py $BA > $O/d_${w}_$r.log 2>&1 || { tail -5 $O/d_${w}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/d_${w}_$r.log') if l.startswith('{')][-1]); x=d['delivered']
print('wgs $w $r', round(d['value']/1e6,2), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3), 'ms', round(x['pcie_GBps'],1), 'GB/s', x['checked_last_step_from_host_memory']['msc_equal_transmitted'], x['checked_last_step_from_host_memory']['fic_blocks_equal_transmitted'])"
done; done
