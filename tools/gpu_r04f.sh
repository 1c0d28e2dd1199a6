#!/bin/bash
# Round 4: GPU suite (packed MSC output, background re-acquisition, display feeds, CFO NCO
# parity), then the driver's bench command with the new legs (delivered, sync loss).
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "suite rc=$?"; grep -E "FAILED|ERROR|passed|failed" $O/gpu_tests.log | tail -8
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04f/bench_c3.log") if l.startswith("{")][-1])
print("value", d["value"] / 1e6, "ms", d["ms_per_step"], "hbm_frac_step", d.get("hbm_frac_step"))
print("delivered", d.get("delivered_symbols_per_s"), json.dumps(d.get("delivered"))[:600])
print("sync_loss", json.dumps(d.get("sync_loss"))[:900])
print("alone", d["kernel_ms_per_launch_alone"], "pipe", d["kernel_ms_per_launch"])
PY
