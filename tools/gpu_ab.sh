#!/bin/bash
# same-box A/B over (library variant, env) pairs on the C3 bench, interleaved REPS times:
#   tools/gpu_ab.sh OUT REPS "lib:ENV=v" ...   (lib = variant name in sdr-j-dab_amd/lib/variants, or "cur")
set -o pipefail
O=gpurun_out/$1; reps=$2; shift 2
mkdir -p $O
L=$(pwd)/sdr-j-dab_amd/lib/variants
for r in $(seq 1 $reps); do
  for spec in "$@"; do
    lib=${spec%%:*}; env=${spec#*:}
    libp=$(pwd)/sdr-j-dab_amd/lib/libdabgpu.so; [ "$lib" != cur ] && libp=$L/libdabgpu_$lib.so
    tag=$(echo "$spec" | tr ':=/ ' '____')
    env DABGPU_LIB=$libp $env timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/${tag}_$r.log 2>&1 || { tail -3 $O/${tag}_$r.log; exit 1; }
    grep '"value"' $O/${tag}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_ms_per_launch']; a=d['kernel_ms_per_launch_alone']
print('%-28s rep $r value %.4g M ms/step %.3f acs %.3f demod %.3f tb %.3f | alone acs %.3f demod %.3f tb %.3f ok=%s' % ('$spec', d['value']/1e6, d['ms_per_step'], k['msc_acs'], k['demod'], k['msc_traceback'], a['msc_acs'], a['demod'], a['msc_traceback'], d['checked_step']['msc_equal_transmitted']))"
  done
done
