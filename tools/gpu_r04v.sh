#!/bin/bash
# Round 4: the DAB+ layer fused into one workgroup per (stream, DAB+ subchannel) (k_dp_layer)
# vs the three-kernel queue form (DABGPU_DP_SPLIT=1).  Parity first (both forms).
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dabplus or c5_full or packed or dropin or gui" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
DABGPU_DP_SPLIT=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dabplus or c5_full" > $O/tests_split.log 2>&1 || { tail -30 $O/tests_split.log; exit 1; }
tail -2 $O/tests_split.log
BA="--workload c5 --steps 20 --warmup 5 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
for r in 1 2; do for v in 0 1; do
  DABGPU_DP_SPLIT=$v timeout -k 10 300 python3 bench.py $BA > $O/c5_${v}_$r.log 2>&1 || { tail -5 $O/c5_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c5 split=$v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'demod', round(k['demod'],3), 'acs', round(k['msc_acs'],3), d['dabplus_last_step'])"
done; done
