#!/bin/bash
# Round 5, call h: C3 tiles-per-workgroup sweep over launch shapes (the knob).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256,128,64,32,16 --slices 1,2,4,8 --tiles 1,2,3,4,6,8 > $OUT/sweep.log 2> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --geom 64,16 --stripes 256,16 --slices 1,8 --tiles 1,2,4,8 > $OUT/sweep16.log 2>> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
python3 -c "
import json
for f in ('$OUT/sweep.log','$OUT/sweep16.log'):
    for l in open(f):
        d=json.loads(l); print(d['geom'], d['stripes'], d['ranks'], d['tiles'], d['ms'], d['frac'])"
