#!/bin/bash
# Round 4: the DAB+ layer on a stream of its own (the run after next's ACS no longer queues
# behind it; its traceback waits) -- DAB+ / fetch / drop-in tests, then C5 and C3 benches.
set -o pipefail
O=gpurun_out/${OUT:-r04ae}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -v --timeout 300 --timeout-method thread -k "dabplus or compact or c5_full or dropin or gui or fetch or packed or solo or au" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --sync-loss-steps 0 > $O/c5_$r.log 2>&1 || { tail -5 $O/c5_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_$r.log') if l.startswith('{')][-1]); x=d['delivered']; k=d['kernel_ms_per_launch']
print('c5 $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), 'acs', round(k['msc_acs'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), round(x['ms_per_step'],3), x['checked_last_step_from_host_memory']['msc_equal_transmitted'], d['dabplus_last_step'])"
done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/c3.log') if l.startswith('{')][-1])
print('c3', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2))"
