#!/bin/bash
# Round 4: (1) PCIe D2H ceiling of the box; (2) C5 kernel stats (rocprofv3) with packed MSC;
# (3) C3 bench, MSC output bits vs packed, interleaved; (4) the sync-loss leg with the
# acquisition wave at priority 3.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/d2h_bw.py 256 > $O/d2h.log 2>&1; cat $O/d2h.log | tail -2
BA="--no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 -- python3 bench.py --workload c5 --steps 10 --warmup 3 --solo-steps 0 $BA --msc-format packed > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
find $O/prof_c5 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/c5_kernel_stats.csv; head -12 $O/c5_kernel_stats.csv | cut -c1-160
for r in 1 2; do for fmt in bits packed; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $BA --msc-format $fmt > $O/c3_${fmt}_$r.log 2>&1 || { tail -5 $O/c3_${fmt}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${fmt}_$r.log') if l.startswith('{')][-1])
print('c3 $fmt $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'tb pipe', round(d['kernel_ms_per_launch']['msc_traceback'],3), 'alone', round(d['kernel_ms_per_launch_alone']['msc_traceback'],3), 'ok', d['checked_step']['msc_equal_transmitted'])"
done; done
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 8 > $O/c3_loss.log 2>&1 || { tail -5 $O/c3_loss.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/c3_loss.log') if l.startswith('{')][-1])
print('loss', json.dumps(d['sync_loss']))"
