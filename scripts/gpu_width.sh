#!/bin/bash
# LDS tile width A/B (RS_UNIT_WIDTH=wide: 128-byte tiles, narrow: 64-byte) for C4 / C5 kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/width
: > gpurun_out/width/times.log
for w in wide narrow; do
  RS_UNIT_WIDTH=$w timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/width/$w -o run -- python3 scripts/time_ops.py --configs C4,C5,C5x8 --iters 30 --tag $w > gpurun_out/width/$w.out 2> gpurun_out/width/$w.err
  rc=$?; [ $rc -eq 0 ] || { echo "fail $w rc=$rc"; tail -5 gpurun_out/width/$w.err; exit $rc; }
  python3 - "$w" >> gpurun_out/width/times.log <<'PY'
import csv, glob, sys
m = sys.argv[1]
f = glob.glob(f"gpurun_out/width/{m}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "_lds" in r["Name"]:
        print(m, r["Name"][40:110], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
cat gpurun_out/width/times.log
