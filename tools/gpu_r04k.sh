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
# PMC: HBM traffic (FETCH_SIZE, WRITE_SIZE) and the SQ pass (VALU, LDS bank conflicts)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
BENCH_ARGS="--solo-steps 0 --delivered-steps 0 --sync-loss-steps 0" $R/tools/pmc_passes.sh r04k/pmc3 "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" > $R/$O/pmc3.log 2>&1 || { tail -5 $R/$O/pmc3.log; exit 1; }
python3 $R/tools/pmc_summary.py $(find $R/$O/pmc3/p3 -name '*counter_collection.csv') > $R/$O/pmc_sq.txt
grep -A9 "k_demod_wg<true, true>" $R/$O/pmc_sq.txt
# C5: DAB+ layer with batched window loads (product) vs the previous layer (cf9edda), interleaved
cd $R
for r in 1 2; do for v in cur dpold; do
  L=sdr-j-dab_amd/lib/libdabgpu.so; [ $v = dpold ] && L=sdr-j-dab_amd/lib/variants/libdabgpu_dpold.so
  DABGPU_LIB=$L timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0 > $O/c5_${v}_$r.log 2>&1 || { tail -5 $O/c5_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c5 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'demod', round(k['demod'],3), 'acs', round(k['msc_acs'],3), 'tb', round(k['msc_traceback'],3), 'sf', d['dabplus_last_step'])"
done; done
