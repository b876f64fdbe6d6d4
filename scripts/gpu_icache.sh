#!/bin/bash
# Instruction-fetch counters of the C3 bench (one --pmc pass, SQ/SQC block).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS} --output-format csv -d gpurun_out/icache -o run -- python3 bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/icache.json 2> gpurun_out/icache.err
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/icache.err; exit $rc; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob("gpurun_out/icache/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_encode_hp" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k[:60], {c: round(v / max(1, n[(k, c)] / 1), 1) for c, v in d.items()})
PY
