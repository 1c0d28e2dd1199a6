#!/bin/bash
# Round 4: k_acquire with the 64-sample group (lane 0 runs the two chains, the 64 lanes
# test side by side) and the sLevel step unfused -- full GPU suite, then the sync-loss leg
# and the kernel's own time.
set -o pipefail
O=gpurun_out/r04aa; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); s=d['sync_loss']
print('C3', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'acquire_ms', d.get('acquire_ms'), 'sync', json.dumps(s)[:600])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o c3 -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
f=$(find $R/$O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $R/$O/c3_kernel_stats.csv; grep -E "k_acquire" $R/$O/c3_kernel_stats.csv | cut -c1-40,100-220
