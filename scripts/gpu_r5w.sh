#!/bin/bash
# Round 5, call w: bench line with the device record and the copy calibration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5w; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-host > $OUT/bench.json 2> $OUT/bench.err; rc=$?
python3 -c "
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d['device'], d['calibration'], d['other_workloads']['C4_reconstruct']['frac'])" || tail -5 $OUT/bench.err
exit $rc
