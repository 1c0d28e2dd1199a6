#!/bin/bash
# The delivered leg: copies behind the decoding (dabgpu_pipe_fetch, the default) against the
# decoders writing pinned host memory directly (--delivered-mode direct), interleaved.
#   tools/delivered_mode_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
mkdir -p gpurun_out/$O
A="--steps 8 --warmup 2 --no-cpu-baseline --solo-steps 0 --sync-loss-steps 0 --c5-steps 0"
for r in $(seq 1 $REPS); do
    for m in direct fetch; do
        timeout -k 10 240 python3 bench.py $A --delivered-mode $m > gpurun_out/$O/bench_${m}_$r.log 2>&1 || { tail -5 gpurun_out/$O/bench_${m}_$r.log; exit 1; }
        grep '"value"' gpurun_out/$O/bench_${m}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); v=d['delivered']
print('$m rep $r value %.4g M ms/step %.3f | delivered %.4g M ms/step %.3f GB/s %.2f mode %s check %s' % (d['value']/1e6, d['ms_per_step'], d['delivered_symbols_per_s']/1e6, v['ms_per_step'], v['pcie_GBps'], v['mode'], v['checked_last_step_from_host_memory']['msc_equal_transmitted']))" | tee -a gpurun_out/$O/ab.txt
    done
done
