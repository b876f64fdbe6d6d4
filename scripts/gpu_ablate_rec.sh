#!/bin/bash
# Time C4 / C5 for each library under build/ablate/ (LDS-resident kernels)
# under rocprofv3 kernel-trace: per-kernel average durations, one line per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abrec
: > gpurun_out/ablate_rec.log
for d in build/ablate/*/; do
  n=$(basename $d); [ "$n" = common ] && continue
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abrec/$n -o run -- python3 scripts/time_ops.py --configs ${CONFIGS:-C4,C5} --iters 30 --tag $n > gpurun_out/abrec/$n.out 2> gpurun_out/abrec/$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 gpurun_out/abrec/$n.err; exit $rc; }
  python3 - "$n" >> gpurun_out/ablate_rec.log <<'PY'
import csv, glob, sys
n = sys.argv[1]
f = glob.glob(f"gpurun_out/abrec/{n}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_rec_lds" in r["Name"] or "k_enc_lds" in r["Name"]:
        print(n, r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
cat gpurun_out/ablate_rec.log
