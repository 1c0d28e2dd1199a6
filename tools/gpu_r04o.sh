#!/bin/bash
# Round 4: DAB+ layer -- GF tables copied with every load in flight, syndromes of a
# power-of-two RSDims reduced by lane shuffles instead of LDS atomics.  Parity, then C5
# interleaved against the previous layer (HEAD before the change: dpprev).
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dabplus or rs_decode or c5_full or packed" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for v in cur dpprev; do
  L=sdr-j-dab_amd/lib/libdabgpu.so; [ $v = dpprev ] && L=sdr-j-dab_amd/lib/variants/libdabgpu_dpprev.so
  DABGPU_LIB=$L timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0 > $O/c5_${v}_$r.log 2>&1 || { tail -5 $O/c5_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c5 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'demod', round(k['demod'],3), 'acs', round(k['msc_acs'],3), 'tb', round(k['msc_traceback'],3), 'sf', d['dabplus_last_step'])"
done; done
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof5 -o c5 -- python3 $R/bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 --sync-loss-steps 0 > $R/$O/prof5.log 2>&1 || { tail -5 $R/$O/prof5.log; exit 1; }
f=$(find $R/$O/prof5 -name "*kernel_stats.csv" | head -1); cp "$f" $R/$O/c5_kernel_stats.csv; grep "dp_" $R/$O/c5_kernel_stats.csv | cut -c1-120
