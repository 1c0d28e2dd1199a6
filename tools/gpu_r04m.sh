#!/bin/bash
# Round 4: deferred traceback (DABGPU_DEFER_TB=1: run r's traceback queued behind run r+1's
# ACS instead of beside run r+1's demod) with the register-ring traceback and the LDS-DMA
# ones (TB_DMA=1/2 builds, DABGPU_TB_WAVES grid caps).  Parity with deferral first.
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
export TMPDIR=/tmp
DABGPU_DEFER_TB=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pipeline or c3_full or c5_full or packed or dropin or gui" > $O/tests_defer.log 2>&1 || { tail -30 $O/tests_defer.log; exit 1; }
tail -2 $O/tests_defer.log
DABGPU_DEFER_TB=1 DABGPU_TB_WAVES=256 DABGPU_LIB=sdr-j-dab_amd/lib/variants/libdabgpu_tbdma1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c3_full or packed or background" > $O/tests_defer_dma.log 2>&1 || { tail -30 $O/tests_defer_dma.log; exit 1; }
tail -2 $O/tests_defer_dma.log
BA="--steps 10 --warmup 3 --no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
for r in 1 2; do for v in cur defer dma2_0 dma2_256 dma2_512 dma1_256; do
  L=sdr-j-dab_amd/lib/libdabgpu.so; W=0; D=1
  case $v in cur) D=0;; dma2_*) L=sdr-j-dab_amd/lib/variants/libdabgpu_tbdma1.so; W=${v#*_};; dma1_*) L=sdr-j-dab_amd/lib/variants/libdabgpu_tbdma.so; W=${v#*_};; esac
  DABGPU_DEFER_TB=$D DABGPU_TB_WAVES=$W DABGPU_LIB=$L timeout -k 10 300 python3 bench.py $BA > $O/c3_${v}_$r.log 2>&1 || { tail -5 $O/c3_${v}_$r.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c3_${v}_$r.log') if l.startswith('{')][-1]); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('c3 $v $r', round(d['value']/1e6,2), round(d['ms_per_step'],3), 'demod', round(k['demod'],3), round(a['demod'],3), 'acs', round(k['msc_acs'],3), round(a['msc_acs'],3), 'tb', round(k['msc_traceback'],3), round(a['msc_traceback'],3), 'ok', d['checked_step']['msc_equal_transmitted'])"
done; done
