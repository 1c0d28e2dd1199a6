#!/bin/bash
# Round 4: the CFO NCO soft-value test on the round-3 library (exact per-sample table) and on
# the product (double recurrence), then the background re-acquisition test and the bench.
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
L=$(pwd)/sdr-j-dab_amd/lib
for v in r3 cur; do
  lib=$L/libdabgpu.so; [ $v != cur ] && lib=$L/variants/libdabgpu_$v.so
  DABGPU_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "demod_nco" -s -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1
  echo "$v rc=$?"; grep -E "^worst|worst \|" $O/t_$v.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pipeline_oracle.py -k "background or packed or bounds" -s -v --timeout 200 --timeout-method thread > $O/t_bg.log 2>&1
echo "bg rc=$?"; grep -E "background re-acq|stream [01]|PASS|FAIL" $O/t_bg.log | head
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04g/bench_c3.log") if l.startswith("{")][-1])
print("value", d["value"] / 1e6, "ms", d["ms_per_step"], "hbm_frac_step", d.get("hbm_frac_step"))
print("delivered", d.get("delivered_symbols_per_s"), json.dumps(d.get("delivered"))[:700])
print("sync_loss", json.dumps(d.get("sync_loss"))[:1200])
print("alone", d["kernel_ms_per_launch_alone"], "pipe", d["kernel_ms_per_launch"])
PY
for fmt in bits packed; do
  timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --delivered-steps 0 \
      --sync-loss-steps 0 --msc-format $fmt > $O/bench_c5_$fmt.log 2>&1 || { tail -5 $O/bench_c5_$fmt.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/bench_c5_$fmt.log') if l.startswith('{')][-1])
print('c5 $fmt', d['value']/1e6, d['ms_per_step'], 'pipe', d['kernel_ms_per_launch'], 'alone', d['kernel_ms_per_launch_alone'], d['dabplus_last_step'], d['checked_step']['msc_equal_transmitted'])"
done
