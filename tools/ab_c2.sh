#!/bin/bash
# A/B of two builds of libdabgpu.so on the FIC-only workload (the demod dominates):
# tools/ab_c2.sh LIB_A LIB_B -- per-launch k_demod_wg durations from rocprofv3 kernel traces
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
    n=$(basename "$v" .so)
    cp "$v" sdr-j-dab_amd/lib/libdabgpu.so
    timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/ab_$n -o kt --output-format csv -- \
        python3 bench.py --workload c2 --no-cpu-baseline --steps 6 > gpurun_out/ab_$n.log 2>&1
    python3 - "$n" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/ab_{sys.argv[1]}/**/kt_kernel_trace.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    if "demod" in k or "prs_sync" in k or "acs" in k:
        v = sorted(v)
        print(sys.argv[1], k, "n", len(v), "median_us", v[len(v) // 2], "min", v[0])
PY
    grep '"value"' gpurun_out/ab_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms_per_step', d['ms_per_step'])"
done
