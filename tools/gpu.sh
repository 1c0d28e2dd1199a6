#!/bin/bash
# One driver for every GPU-box measurement of this repo (replaces the per-experiment
# gpu_r0* scripts of rounds 3-4).  One step per invocation; chain steps with && in the
# gpurun command so that the first failure ends the call.  Output: gpurun_out/OUT/.
#
#   tools/gpu.sh OUT tests [pytest args...]        -m gpu tests (default: the whole suite)
#   tools/gpu.sh OUT smoke                         __graft_entry__.smoke()
#   tools/gpu.sh OUT bench NAME [bench args...]    python bench.py ... > bench_NAME.log (+ a one-line summary)
#   tools/gpu.sh OUT stats NAME [bench args...]    rocprofv3 --kernel-trace --stats of that bench command
#   tools/gpu.sh OUT pmc NAME "CTRS" [bench args...]  one rocprofv3 --pmc pass (counter limits per pass:
#                                                  MI355X_MICROARCH.md) over a short bench command
#   tools/gpu.sh OUT py NAME script.py [args...]   any python script, output to py_NAME.log
#
# DABGPU_LIB=path selects another build of libdabgpu.so (A/B variants), as dabamd reads it.
set -o pipefail
OUT=$1; STEP=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/$OUT
mkdir -p "$O"
export TMPDIR=/tmp

summary() {   # the bench line's headline numbers
    python3 - "$1" <<'EOF'
import json, sys
ls = [l for l in open(sys.argv[1]) if l.startswith("{")]
if not ls:
    sys.exit(0)
d = json.loads(ls[-1])
k = d.get("kernel_ms_per_launch", {}); a = d.get("kernel_ms_per_launch_alone", {})
print("value %.2f M  ms/step %.3f  acs %.3f (alone %.3f)  demod alone %.3f  tb alone %.3f  checked %s" % (
    d["value"] / 1e6, d["ms_per_step"], k.get("msc_acs", 0), a.get("msc_acs", 0), a.get("demod", 0),
    a.get("msc_traceback", 0), d.get("checked_step", {}).get("msc_equal_transmitted") if isinstance(
        d.get("checked_step"), dict) else [c["msc_equal_transmitted"] for c in d["checked_step"]]))
for key in ("c4_fed", "delivered_symbols_per_s"):
    if key in d:
        print(key, d[key] if not isinstance(d[key], dict) else {x: d[key][x] for x in list(d[key])[:6]})
EOF
}

case $STEP in
tests)
    [ $# -eq 0 ] && set -- tests
    timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/tests.log 2>&1
    rc=$?; tail -3 $O/tests.log; exit $rc ;;
smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    rc=$?; tail -2 $O/smoke.log; exit $rc ;;
bench)
    NAME=$1; shift
    timeout -k 10 600 python3 -u bench.py "$@" > $O/bench_$NAME.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench_$NAME.log; exit $rc; }
    echo "bench $NAME: $(summary $O/bench_$NAME.log)"; exit 0 ;;
stats)
    NAME=$1; shift
    cd /tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats_$NAME -o s --output-format csv \
        -- python3 $R/bench.py "$@" > $O/stats_$NAME.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/stats_$NAME.log; exit $rc; }
    f=$(find $O/stats_$NAME -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && head -12 "$f"; exit 0 ;;
pmc)
    NAME=$1; CTRS=$2; shift 2
    cd /tmp
    timeout -s KILL 180 rocprofv3 --pmc $CTRS --kernel-trace -d $O/pmc_$NAME -o p --output-format csv \
        -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --solo-steps 0 --delivered-steps 0 \
        --sync-loss-steps 0 "$@" > $O/pmc_$NAME.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -8 $O/pmc_$NAME.log; exit $rc; }
    python3 $R/tools/pmc_summary.py $(find $O/pmc_$NAME -name '*counter_collection.csv') > $O/pmc_$NAME.txt
    echo "pmc $NAME: $(wc -l < $O/pmc_$NAME.txt) summary lines"; exit 0 ;;
py)
    NAME=$1; shift
    timeout -k 10 600 python3 -u "$@" > $O/py_$NAME.log 2>&1
    rc=$?; tail -15 $O/py_$NAME.log; exit $rc ;;
*)
    echo "unknown step $STEP"; exit 2 ;;
esac
