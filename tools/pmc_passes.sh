#!/bin/bash
# PMC passes over one short bench run, one rocprofv3 process per pass (counter
# limits per pass: MI355X_MICROARCH.md).  usage: tools/pmc_passes.sh OUTDIR "CTRS1" "CTRS2" ...
# Each pass: gpurun_out/OUTDIR/pN/*_counter_collection.csv
out=$1; shift
cd /tmp && export TMPDIR=/tmp
root=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $root/gpurun_out/$out
i=0
for ctrs in "$@"; do
    i=$((i+1))
    echo "[pmc pass $i] $ctrs"
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace -d $root/gpurun_out/$out/p$i -o p$i --output-format csv \
        -- python3 $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $root/gpurun_out/$out/p$i.log 2>&1
    rc=$?
    echo "[pmc pass $i] rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $root/gpurun_out/$out/p$i.log; exit $rc; }
done
exit 0
