#!/bin/bash
# Round 4 final-build measurements: driver command (C3), C5 bench, C5 HBM traffic passes.
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('C3', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), 'roof', round(d['roofline']['frac'],3), round(d['roofline']['frac_of_ceiling'],3), d['roofline']['traffic'] is not None, 'demod', round(d['roofline_hbm_demod']['frac'],3), round(d['roofline_hbm_demod']['frac_alone'],3), 'cpu', round(d['cpu_baseline']['value']), 'sync', round(d['sync_loss']['async']['hit_ms_per_loss'],3), round(d['hbm_frac_step'],3), d['checked_step']['msc_equal_transmitted'])"
timeout -k 10 400 python3 bench.py --workload c5 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_c5.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('C5', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'delivered', round(d['delivered_symbols_per_s']/1e6,2), 'cpu', round(d['cpu_baseline']['value']), d['dabplus_last_step'])"
cd /tmp
BENCH_ARGS="--workload c5 --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0" $R/tools/pmc_passes.sh r04t/pmc5 "FETCH_SIZE" "WRITE_SIZE" > $R/$O/pmc5.log 2>&1 || { tail -5 $R/$O/pmc5.log; exit 1; }
python3 $R/tools/pmc_traffic.py $(find $R/$O/pmc5/p1 -name '*counter_collection.csv') $(find $R/$O/pmc5/p2 -name '*counter_collection.csv') $R/$O/traffic_c5.json | grep -E "acs2|demod_wg<true, true, true>|traceback2|dp_"
