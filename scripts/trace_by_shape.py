"""Average rocprofv3 --kernel-trace durations per (kernel, grid shape): the
--stats csv averages a kernel over every launch shape it ran with."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/run_kernel_trace.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        gx = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        gy = r.get("Grid_Size_Y") or "1"
        key = (r["Kernel_Name"][:60], int(gx), int(gy))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, gx, gy), v in sorted(agg.items()):
    print(f"{k:60s} grid {gx:8d} x {gy:3d} launches {len(v):4d} avg {sum(v)/len(v):10.2f} us")
