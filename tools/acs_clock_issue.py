"""Achieved clock and VALU issue utilisation of a kernel from one rocprofv3 --pmc pass
(tools/gpu.sh OUT pmc NAME "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY
SQ_INSTS_VALU"), per dispatch and for the largest (full-batch) dispatch:

  clock_ghz            = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md,
                         DVFS give-back: rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs)
  valu_issue_utilisation = 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8):
                         the share of each SIMD's cycles in which a wave issued a VALU
                         instruction (SQ_ACTIVE_INST_* count quad-cycles)
  cycles_per_valu      = 4 x SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU
  wait_inst / wait_any / active_any = SQ_WAIT_INST_ANY, SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY
                         over SQ_WAVE_CYCLES (per wave, disjoint)

usage: python tools/acs_clock_issue.py PMC_DIR KERNEL_SUBSTRING > profiles/rNN_acs_clock_issue.json
"""
import csv
import glob
import json
import os
import sys


def main(d, kname):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    tr = {r["Dispatch_Id"]: r for r in csv.DictReader(open(kt))}
    by = {}
    name = None
    for r in csv.DictReader(open(cc)):
        if kname in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("(")[0]
            by.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = []
    for disp, c in sorted(by.items(), key=lambda x: int(x[0])):
        t = tr[disp]
        dur = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) * 1e-9
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        rows.append({"dispatch": int(disp), "ms": dur * 1e3, "clock_ghz": cyc / dur / 1e9,
                     "valu_issue_utilisation": 4 * c["SQ_ACTIVE_INST_VALU"] / (1024 * cyc),
                     "cycles_per_valu": 4 * c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"],
                     "valu_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
                     "wait_inst": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
                     "wait_any": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
                     "active_any": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]})
    full = [r for r in rows if r["ms"] >= 0.5 * max(x["ms"] for x in rows)]
    out = {"kernel": name, "source": d, "dispatches": rows}
    for k in ("clock_ghz", "valu_issue_utilisation", "cycles_per_valu", "wait_inst", "wait_any", "active_any"):
        out[k] = sum(r[k] for r in full) / len(full)
    out["note"] = ("mean over the full-batch dispatches of one profiled bench run (profiled passes run a few % "
                   "slower than unprofiled ones, MI355X_MICROARCH.md DVFS item 2)")
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
