#!/bin/bash
# Round 4: the demod's soft-bit stage in bank-spread carrier pairs (stage_layout.h) --
# parity (demod soft bits, pipeline), same-box A/B against the previous layout
# (variants/libdabgpu_base.so), and an SQ pass for the LDS bank conflicts.
set -o pipefail
O=gpurun_out/r04al; mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
V=$R/sdr-j-dab_amd/lib/variants/libdabgpu_base.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for v in base new; do
  if [ $v = base ]; then export DABGPU_LIB=$V; else unset DABGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sync-loss-steps 0 --delivered-steps 0 > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod alone', round(a['demod'],3), 'acs', round(k['msc_acs'],3), d['checked_step']['msc_equal_transmitted'])"
done; done
unset DABGPU_LIB
cd /tmp
BENCH_ARGS="--solo-steps 0 --delivered-steps 0 --sync-loss-steps 0" $R/tools/pmc_passes.sh r04al/pmc "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" > $R/$O/pmc.log 2>&1 || { tail -5 $R/$O/pmc.log; exit 1; }
python3 $R/tools/pmc_summary.py $(find $R/$O/pmc/p1 -name '*counter_collection.csv') > $R/$O/pmc_sq.txt
grep -A9 "k_demod_wg<true, true, true>" $R/$O/pmc_sq.txt | grep -E "void|VALU|LDS_BANK|LDS_IDX"
