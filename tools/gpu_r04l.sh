#!/bin/bash
# Round 4: LDS-DMA traceback (TB_DMA=1: two 16 KB LDS images filled by global_load_lds_dwordx4,
# decision columns XOR-swizzled by codeword row, 56 VGPRs) vs the register-ring traceback
# (256 VGPRs + 84 AGPRs).  Parity of the variant first (Viterbi operators + pipeline), then
# the C3 bench interleaved.
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
V=sdr-j-dab_amd/lib/variants/libdabgpu_tbdma.so
DABGPU_TB_WAVES=256 DABGPU_LIB=$V timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread -k "viterbi or profile or c3_full or c5_full or packed or dabplus or fic or au_layouts" > $O/tests_tbdma.log 2>&1 || { tail -30 $O/tests_tbdma.log; exit 1; }
tail -2 $O/tests_tbdma.log
DABGPU_LIB=sdr-j-dab_amd/lib/variants/libdabgpu_tbdma1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread -k "viterbi or c3_full or packed" > $O/tests_tbdma1.log 2>&1 || { tail -30 $O/tests_tbdma1.log; exit 1; }
tail -2 $O/tests_tbdma1.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_dropin.log 2>&1 || { tail -30 $O/tests_dropin.log; exit 1; }
tail -2 $O/tests_dropin.log
BA="--steps 10 --warmup 3 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
for r in 1; do for v in cur tbdma tbdma_256 tbdma_512 tbdma1 tbdma1_256 tbdma1_512; do
  L=sdr-j-dab_amd/lib/variants/libdabgpu_${v%_*}.so; W=${v#*_}; [ "$W" = "$v" ] && W=0
  [ $v = cur ] && L=sdr-j-dab_amd/lib/libdabgpu.so
  DABGPU_TB_WAVES=$W DABGPU_LIB=$L timeout -k 10 300 python3 bench.py $BA > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), round(a['demod'],3), 'acs', round(k['msc_acs'],3), round(a['msc_acs'],3), 'tb', round(k['msc_traceback'],3), round(a['msc_traceback'],3), 'ok', d['checked_step']['msc_equal_transmitted'])"
done; done
# C5 with the batched DAB+ window loads (both libraries carry them)
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c5 $BA > $O/c5_$r.log 2>&1 || { tail -5 $O/c5_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c5 $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'dabplus', round(k['dabplus'],3), round(a['dabplus'],3), 'sf', d['dabplus_last_step'])"
done
