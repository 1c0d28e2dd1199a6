"""Summarise rocprofv3 counter_collection.csv files: per kernel name, the mean of
each counter over its dispatches (largest dispatch group per kernel name)."""
import collections
import csv
import sys

def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(agg.items()):
        if k.startswith("__amd"):
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} n={len(v):3d} mean={sum(v)/len(v):.4g} max={max(v):.4g}")

if __name__ == "__main__":
    main(sys.argv[1:])
