"""Per-run mean of every PMC counter of one kernel: rocprofv3 --pmc output
dirs named <prefix>_<config>_<pass> -> one row per config.
usage: pmc_by_run.py DIR KERNEL_SUBSTRING"""
import collections
import csv
import glob
import os
import re
import sys

root, pat = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/pmc_*/**/run_counter_collection.csv", recursive=True)):
    run = os.path.relpath(f, root).split(os.sep)[0]
    cfg = re.sub(r"^pmc_|_\d+$", "", run)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[cfg][r["Counter_Name"]].append(float(r["Counter_Value"]))
for cfg, cs in agg.items():
    print(cfg)
    for c, v in sorted(cs.items()):
        print(f"  {c:40s} n={len(v):3d} mean={sum(v) / len(v):.5g}")
