#!/bin/bash
# Round 4 final build: full -m gpu suite, smoke, the driver's bench command, C5 bench,
# C3 kernel stats (rocprofv3).
set -o pipefail
O=gpurun_out/${OUT:-r04fin}; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('C3', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), 'roof', round(d['roofline']['frac'],3), round(d['roofline']['frac_of_ceiling'],3), 'demod', round(d['roofline_hbm_demod']['frac'],3), round(d['roofline_hbm_demod']['frac_alone'],3), 'cpu', round(d['cpu_baseline']['value']), 'acq', round(d['acquire_ms']['ms'],2), 'sync', round(d['sync_loss']['sync']['hit_ms_per_loss'],1), round(d['sync_loss']['async']['hit_ms_per_loss'],3), round(d['hbm_frac_step'],3), d['checked_step']['msc_equal_transmitted'])"
timeout -k 10 400 python3 bench.py --workload c5 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_c5.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('C5', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), 'cpu', round(d['cpu_baseline']['value']), d['dabplus_last_step'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o c3 -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 --delivered-steps 0 > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
f=$(find $R/$O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $R/$O/c3_kernel_stats.csv; cut -c1-120 $R/$O/c3_kernel_stats.csv | head -6
