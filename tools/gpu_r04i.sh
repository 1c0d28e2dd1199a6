#!/bin/bash
# Round 4: the null search alone (tools/acq_bench.py), previous build (acq0) vs the block
# loads issued together (cur); C5 kernel stats in CSV.
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
L=$(pwd)/sdr-j-dab_amd/lib
for v in acq0 cur; do
  lib=$L/libdabgpu.so; [ $v != cur ] && lib=$L/variants/libdabgpu_$v.so
  for args in "--ensembles 64" "--ensembles 1" "--ensembles 1 --jam" "--ensembles 64 --jam"; do
    DABGPU_LIB=$lib timeout -k 10 200 python3 tools/acq_bench.py $args > $O/acq.log 2>&1 || { tail -5 $O/acq.log; exit 1; }
    echo "$v $(tail -1 $O/acq.log)"
  done
done
BA="--no-cpu-baseline --delivered-steps 0 --sync-loss-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --workload c5 --steps 10 --warmup 3 --solo-steps 0 $BA --msc-format packed > $O/prof_c5.log 2>&1 || { tail -5 $O/prof_c5.log; exit 1; }
f=$(find $O/prof_c5 -name "*kernel_stats.csv" | head -1); cp "$f" $O/c5_kernel_stats.csv; cut -c1-150 $O/c5_kernel_stats.csv | head -14
