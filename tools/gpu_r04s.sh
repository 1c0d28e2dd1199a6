#!/bin/bash
# Round 4 profiles of the RING8 build: C3 kernel trace + timeline, HBM traffic (FETCH_SIZE,
# WRITE_SIZE) and the SQ pass; C5 kernel stats.
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o c3 -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --solo-steps 0 --delivered-steps 0 > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
f=$(find $R/$O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $R/$O/c3_kernel_stats.csv; cut -c1-110 $R/$O/c3_kernel_stats.csv | head -8
t=$(find $R/$O/prof -name "*kernel_trace.csv" | head -1); python3 $R/tools/trace_timeline.py "$t" --steps 3 > $R/$O/timeline.txt 2>&1; tail -24 $R/$O/timeline.txt
BENCH_ARGS="--solo-steps 0 --delivered-steps 0 --sync-loss-steps 0" $R/tools/pmc_passes.sh r04s/pmc3 "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" > $R/$O/pmc3.log 2>&1 || { tail -5 $R/$O/pmc3.log; exit 1; }
python3 $R/tools/pmc_traffic.py $(find $R/$O/pmc3/p1 -name '*counter_collection.csv') $(find $R/$O/pmc3/p2 -name '*counter_collection.csv') $R/$O/traffic_c3.json | grep -E "acs2|demod_wg<true, true>|traceback2"
python3 $R/tools/pmc_summary.py $(find $R/$O/pmc3/p3 -name '*counter_collection.csv') > $R/$O/pmc_sq.txt
grep -A9 "k_demod_wg<true, true, true>\|k_acs2<3, 2, true>" $R/$O/pmc_sq.txt | grep -E "void|VALU|LDS_BANK|LDS_IDX"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof5 -o c5 -- python3 $R/bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0 > $R/$O/prof5.log 2>&1 || { tail -5 $R/$O/prof5.log; exit 1; }
f=$(find $R/$O/prof5 -name "*kernel_stats.csv" | head -1); cp "$f" $R/$O/c5_kernel_stats.csv
