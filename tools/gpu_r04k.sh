#!/bin/bash
# Round 4 checkpoint: the whole -m gpu suite, the driver's bench command (packed MSC by
# default), and a kernel trace of the C3 main leg for the round's kernel stats + timeline.
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 --delivered-steps 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -c1-120 "$f" | head -14
t=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 tools/trace_timeline.py "$t" --steps 3 > $O/timeline.txt 2>&1; tail -60 $O/timeline.txt
