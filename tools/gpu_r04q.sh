#!/bin/bash
# Round 4 checkpoint 2: the whole -m gpu suite, the driver's bench command, C5 bench.
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('C3', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), 'roof', round(d['roofline']['frac'],3), 'demod', round(d['roofline_hbm_demod']['frac'],3), round(d['roofline_hbm_demod']['frac_alone'],3), 'cpu', round(d['cpu_baseline']['value']), 'sync', round(d['sync_loss']['async']['hit_ms_per_loss'],3), d['checked_step']['msc_equal_transmitted'])"
timeout -k 10 400 python3 bench.py --workload c5 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_c5.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('C5', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), 'cpu', round(d['cpu_baseline']['value']), d['dabplus_last_step'])"
