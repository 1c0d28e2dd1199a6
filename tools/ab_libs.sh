#!/bin/bash
# Same-box A/B of library builds on the full bench workload (not part of the product):
#   tools/ab_libs.sh REPS LIB... -- each lib runs `bench.py --steps 8` via DABGPU_LIB,
# libs interleaved REPS times; prints value and in-pipeline k_acs2 / demod / traceback ms.
reps=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $reps); do
  for v in "$@"; do
    n=$(basename "$v" .so)
    DABGPU_LIB=$v timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} \
        > gpurun_out/ab_${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab_${n}_$r.log; exit 1; }
    grep '"value"' gpurun_out/ab_${n}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_launch']
a=d.get('kernel_ms_per_launch_alone') or {}
print('$n rep $r value %.4g M ms/step %.3f acs %.3f demod %.3f tb %.3f dabplus %.3f' % (d['value']/1e6, d['ms_per_step'], k['msc_acs'], k['demod'], k['msc_traceback'], k['dabplus'])
      + (' | alone demod %.3f acs %.3f tb %.3f' % (a['demod'], a['msc_acs'], a['msc_traceback']) if a.get('demod') else ''))"
  done
done
