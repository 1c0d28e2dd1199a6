"""bench.py end to end on a small workload: the driver reads exactly one JSON line from
it, so the line's contract (the keys, the roofline and CPU-baseline blocks' shape, every
leg's checked step) is tested here on a few ensembles and frames rather than discovered
at round end.  The bench runs as a child process (it owns the GPU there)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline")


@pytest.mark.gpu
def test_bench_prints_one_checked_line():
    # (4-frame steps: 6 warm-up steps cover the AFC's convergence under the default 1300 Hz
    # offset, ~11 frames, as the default run's 5 x 24 frames do)
    cmd = [sys.executable, "bench.py", "--ensembles", "4", "--frames", "4", "--steps", "2", "--warmup", "6",
           "--no-cpu-baseline", "--solo-steps", "1", "--delivered-steps", "2", "--sync-loss-steps", "2",
           "--c5-steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 6 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["config"]["ensembles_per_gpu"] == 4 and d["config"]["frames_per_step"] == 4
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert 0 < roof["frac"] < 1
    # every leg decoded ensemble 0 of its step to the transmitted bits
    ck = d["checked_step"]
    assert ck["fic_blocks_equal_transmitted"] and ck["msc_equal_transmitted"] == ck["msc_codewords"] > 0
    dl = d["delivered"]["checked_last_step_from_host_memory"]
    assert dl["fic_blocks_equal_transmitted"] and dl["msc_equal_transmitted"] == dl["msc_codewords"] > 0
    c5 = d["c5"]
    assert "error" not in c5, c5
    c5c = c5["checked_step"]
    assert c5["value"] > 0 and c5c["msc_equal_transmitted"] == c5c["msc_codewords"] > 0
    assert c5c["fic_blocks_equal_transmitted"] and c5c["cif_records"] > 0
    assert "sync_loss" in d
    print("bench line:", {k: d[k] for k in ("value", "ms_per_step")}, "c5", c5["value"])
