#!/bin/bash
# Round 5, call i: C3 tiles per workgroup (1 vs 4 vs 2) against the stripe
# count per launch, full rows, plus 128 stripes on a fresh allocation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5i; mkdir -p $OUT
timeout -k 10 400 python3 scripts/c3_tpw_sweep.py --stripes 320,288,256,224,192,160,128,96 --slices 1 --tiles 1,2,4 > $OUT/sweep.log 2> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --stripes 128 --slices 1 --tiles 1,2,4 > $OUT/sweep128.log 2>> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1 --tiles 1,2,4 > $OUT/sweep256.log 2>> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
python3 -c "
import json
for f in ('$OUT/sweep.log','$OUT/sweep128.log','$OUT/sweep256.log'):
    print(f)
    for l in open(f):
        d=json.loads(l); print(d['stripes'], d['tiles'], d['ms'], d['frac'])"
