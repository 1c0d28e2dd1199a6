#!/bin/bash
# PMC passes over any short command, one rocprofv3 process per pass (counter limits per
# pass: MI355X_MICROARCH.md).  usage: tools/pmc_cmd.sh OUTDIR "CTRS1" ["CTRS2" ...] -- CMD ARGS...
# Each pass: gpurun_out/OUTDIR/pN/*_counter_collection.csv; a failing pass ends the script.
out=$1; shift
passes=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=("$1"); shift; done
shift
root=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
mkdir -p $root/gpurun_out/$out
i=0
for ctrs in "${passes[@]}"; do
    i=$((i+1))
    echo "[pmc pass $i] $ctrs"
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace -d $root/gpurun_out/$out/p$i -o p$i --output-format csv \
        -- "$@" > $root/gpurun_out/$out/p$i.log 2>&1
    rc=$?
    echo "[pmc pass $i] rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $root/gpurun_out/$out/p$i.log; exit $rc; }
done
python3 $root/tools/pmc_summary.py $(find $root/gpurun_out/$out -name '*counter_collection.csv') > $root/gpurun_out/$out/summary.txt
exit 0
