"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE,
separate passes as MI355X_MICROARCH.md's HBM section prescribes).

For each kernel the dispatch with the LARGEST counter value (the full-batch
launch the bench times moves the most bytes) is taken.  FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads, so fetched bytes = 2 x FETCH_SIZE
(calibrated here on k_traceback, whose 16-B/lane reads of the decision words are
known exactly).  Writes are taken as reported.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON
"""
import csv
import json
import sys


def largest(path, counter):
    best = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        g = int(r["Grid_Size"])
        v = float(r["Counter_Value"])
        if k not in best or v > best[k][1]:
            best[k] = (g, v)
    return best


def main(fetch_csv, write_csv, out):
    f = largest(fetch_csv, "FETCH_SIZE")
    w = largest(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        if k.startswith("__amd"):
            continue
        fb = 2.0 * f[k][1] * 1024 if k in f else None
        wb = w[k][1] * 1024 if k in w else None
        res[k] = {"grid": (f.get(k) or w.get(k))[0], "fetch_bytes": fb, "write_bytes": wb,
                  "hbm_bytes": (fb or 0) + (wb or 0)}
    json.dump({"source": [fetch_csv, write_csv], "note": __doc__.strip().splitlines()[0], "kernels": res},
              open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:32s} grid={v['grid']:8d} fetch={v['fetch_bytes'] or 0:12.4g} write={v['write_bytes'] or 0:12.4g}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
