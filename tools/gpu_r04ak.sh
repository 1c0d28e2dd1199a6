#!/bin/bash
# Round 4: C3 timeline of the kept build (demod gated on the ACS).
set -o pipefail
O=gpurun_out/r04ak; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o c3 -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 --delivered-steps 0 > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
t=$(find $R/$O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/trace_timeline.py "$t" --steps 3 > $R/$O/timeline.txt 2>&1; tail -34 $R/$O/timeline.txt
