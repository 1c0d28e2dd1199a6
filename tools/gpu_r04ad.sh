#!/bin/bash
# Round 4: C5 kernel timeline (where a 0.6 ms DAB+ step goes).
set -o pipefail
O=gpurun_out/r04ad; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof5 -o c5 -- python3 $R/bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0 > $R/$O/prof5.log 2>&1 || { tail -5 $R/$O/prof5.log; exit 1; }
t=$(find $R/$O/prof5 -name "*kernel_trace.csv" | head -1); python3 $R/tools/trace_timeline.py "$t" --steps 4 > $R/$O/timeline_c5.txt 2>&1; tail -60 $R/$O/timeline_c5.txt
