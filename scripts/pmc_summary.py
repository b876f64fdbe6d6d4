"""Summarize rocprofv3 PMC csv output dirs: mean counter value per kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:32s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
