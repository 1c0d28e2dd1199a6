"""Kernel timeline of a rocprofv3 --kernel-trace run (rocpd SQLite database or
kernel_trace.csv): per-kernel average durations and, for the last few pipeline
steps, when each kernel ran relative to the step's first front-end launch, on which
stream, and how much of its span overlapped kernels of the other streams.

  python tools/trace_timeline.py gpurun_out/prof/run_results.db [--steps 3] [--stats out.csv]
"""
import argparse
import csv
import sqlite3
from collections import defaultdict


def load(path):
    rows = []
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for name, start, end, stream, grid, wg in db.execute(
                "select name, start, end, stream_id, grid_x, workgroup_x from kernels order by start"):
            rows.append(dict(name=name, start=int(start), end=int(end), stream=stream, grid=grid, wg=wg))
    else:
        for r in csv.DictReader(open(path)):
            rows.append(dict(name=r["Kernel_Name"], start=int(r["Start_Timestamp"]), end=int(r["End_Timestamp"]),
                             stream=r.get("Stream_Id", r.get("Queue_Id")), grid=r.get("Grid_Size_X"),
                             wg=r.get("Workgroup_Size_X")))
    return rows


def short(n):
    n = n.replace("dab::", "").replace("void ", "")
    return n.split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--stats", help="write per-kernel stats CSV here")
    a = ap.parse_args()
    rows = [r for r in load(a.trace) if "rocclr" not in r["name"]]
    agg = defaultdict(list)
    for r in rows:
        agg[short(r["name"])].append(r["end"] - r["start"])
    print(f"{'kernel':42s} {'calls':>6s} {'avg ms':>9s} {'total ms':>10s}")
    out = []
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:42s} {len(v):6d} {sum(v) / len(v) / 1e6:9.3f} {sum(v) / 1e6:10.2f}")
        out.append((k, len(v), sum(v) / len(v) / 1e6, sum(v) / 1e6))
    if a.stats:
        with open(a.stats, "w") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "avg_ms", "total_ms"])
            w.writerows(out)
    # steps: each starts with the front end's big demod launch
    starts = [r["start"] for r in rows if short(r["name"]).startswith("k_demod_wg") and r["grid"] and int(r["grid"]) > 100000]
    if len(starts) < 2:
        return
    print()
    for i in range(max(0, len(starts) - 1 - a.steps), len(starts) - 1):
        t0, t1 = starts[i], starts[i + 1]
        print(f"--- step {i}: {(t1 - t0) / 1e6:.3f} ms")
        for r in rows:
            if r["end"] < t0 or r["start"] >= t1:
                continue
            print(f"  {(r['start'] - t0) / 1e6:8.3f} .. {(r['end'] - t0) / 1e6:8.3f}  ({(r['end'] - r['start']) / 1e6:7.3f})"
                  f"  s{r['stream']}  {short(r['name'])}")


if __name__ == "__main__":
    main()
