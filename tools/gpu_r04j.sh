#!/bin/bash
# Round 4: the delivered leg (dabgpu_pipe_fetch) -- copies on a high-priority stream (product)
# vs on the back-end stream (DABGPU_FETCH_ON_BACK=1), and with HSA_ENABLE_SDMA=1; a
# kernel-trace of the delivered leg shows whether the D2H copies are blit kernels.
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
BA="--steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 --delivered-steps 10"
for r in 1 2; do for v in "X=0" "DABGPU_FETCH_ON_BACK=1" "HSA_ENABLE_SDMA=1"; do
  env $v timeout -k 10 300 python3 bench.py $BA > $O/d_$r.log 2>&1 || { tail -5 $O/d_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/d_$r.log') if l.startswith('{')][-1]); x=d['delivered']
print('$v', round(d['value']/1e6,2), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3), 'ms', round(x['pcie_GBps'],1), 'GB/s', x['checked_last_step_from_host_memory']['msc_equal_transmitted'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o d -- python3 bench.py $BA > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -c1-120 "$f" | head -12
