#!/bin/bash
# The delivered leg with the FIC as FIB bytes (DABGPU_PACK_FIC, bench default) against one
# bit per byte, interleaved; parity tests of the packed FIC first.
#   tools/fic_bytes_ab.sh OUT REPS
set -o pipefail
O=$1; REPS=${2:-3}
mkdir -p gpurun_out/$O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py -x -q -m gpu -k "packed or fetch or compact" \
    --timeout 120 --timeout-method thread > gpurun_out/$O/tests.log 2>&1 || { tail -30 gpurun_out/$O/tests.log; exit 1; }
tail -2 gpurun_out/$O/tests.log
A="--steps 8 --warmup 2 --no-cpu-baseline --solo-steps 0 --sync-loss-steps 0 --c5-steps 0"
for r in $(seq 1 $REPS); do
    for f in bytes bits; do
        timeout -k 10 240 python3 bench.py $A --delivered-fic $f > gpurun_out/$O/bench_${f}_$r.log 2>&1 || { tail -5 gpurun_out/$O/bench_${f}_$r.log; exit 1; }
        grep '"value"' gpurun_out/$O/bench_${f}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); v=d['delivered']
print('$f rep $r value %.4g M ms/step %.3f | delivered %.4g M ms/step %.3f bytes %d GB/s %.2f check %s' % (d['value']/1e6, d['ms_per_step'], d['delivered_symbols_per_s']/1e6, v['ms_per_step'], v['bytes_to_host_per_step'], v['pcie_GBps'], v['checked_last_step_from_host_memory']['msc_equal_transmitted']))" | tee -a gpurun_out/$O/ab.txt
    done
done
