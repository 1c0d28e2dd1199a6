#!/bin/bash
# same-box A/B of library variants (sdr-j-dab_amd/lib/variants/libdabgpu_NAME.so) on the
# C3 bench, interleaved REPS times:  tools/ab_round3.sh REPS NAME...
reps=$1; shift
L=$(pwd)/sdr-j-dab_amd/lib/variants
for r in $(seq 1 $reps); do
  for v in "$@"; do
    DABGPU_LIB=$L/libdabgpu_$v.so timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab3_${v}_$r.log 2>&1 || { tail -3 gpurun_out/ab3_${v}_$r.log; exit 1; }
    grep '"value"' gpurun_out/ab3_${v}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('$v rep $r value %.4g M ms/step %.3f acs %.3f demod %.3f tb %.3f | alone acs %.3f demod %.3f tb %.3f' % (d['value']/1e6, d['ms_per_step'], k['msc_acs'], k['demod'], k['msc_traceback'], a['msc_acs'], a['demod'], a['msc_traceback']))"
  done
done
