#!/bin/bash
# Round 4: compact DAB+ superframe output -- parity (compact vs sparse, drop-ins), then the
# C5 bench with its delivered leg (only the run's superframes cross PCIe).
set -o pipefail
O=gpurun_out/r04z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compact or dabplus or c5_full or dropin or gui or fetch" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --sync-loss-steps 0 > $O/c5_$r.log 2>&1 || { tail -5 $O/c5_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_$r.log') if l.startswith('{')][-1]); x=d['delivered']
print('c5 $r', round(d['value']/1e6,2), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3), round(x['bytes_to_host_per_step']/1e6,2), 'MB', round(x['pcie_GBps'],1), 'GB/s', x['checked_last_step_from_host_memory']['msc_equal_transmitted'])"
done
