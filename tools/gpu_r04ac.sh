#!/bin/bash
# Round 4: dabgpu_pipe_fetch's copies on a stream of their own (the next run's ACS no longer
# queues behind them; its traceback waits) -- fetch/delivery tests, then C3 and C5 with the
# delivered leg.
set -o pipefail
O=gpurun_out/r04ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py tests/test_gpu_dropin.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fetch or compact or packed or dropin or gui" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 > $O/c3_$r.log 2>&1 || { tail -5 $O/c3_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_$r.log') if l.startswith('{')][-1]); x=d['delivered']
print('c3 $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3), round(x['pcie_GBps'],1), 'GB/s', x['checked_last_step_from_host_memory']['msc_equal_transmitted'])"
done
timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --sync-loss-steps 0 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/c5.log') if l.startswith('{')][-1]); x=d['delivered']
print('c5', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3), x['checked_last_step_from_host_memory']['msc_equal_transmitted'])"
