#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit.
# usage: tools/gpu_steps.sh NAME SECONDS CMD... [::: NAME SECONDS CMD...]...
# A step that fails with an ordinary test failure (rc 1, no device fault in its log)
# lets the next step run; any other failure (abort, segfault, timeout, device fault)
# ends the script there.
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
    name=$1; secs=$2; shift 2
    cmd=()
    while [ $# -gt 0 ] && [ "$1" != ":::" ]; do cmd+=("$1"); shift; done
    [ "$1" == ":::" ] && shift
    echo "[step $name] ${cmd[*]}"
    timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "EXIT $rc" >> "gpurun_out/$name.log"
    echo "[step $name] rc=$rc"
    tail -n 3 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then
        if [ $rc -ne 1 ] || grep -qi "illegal memory\|memory access fault\|hipErrorLaunchFailure\|kernel_errors\|device-side" "gpurun_out/$name.log"; then
            echo "[step $name] stopping: rc=$rc"
            exit $rc
        fi
    fi
done
exit 0
