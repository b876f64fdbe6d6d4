#!/bin/bash
# Round 5, call m: C3 per-rank slices (2/4/8-rank byte ranges, 256 stripes):
# tiles per workgroup x tile distance.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5m; mkdir -p $OUT; : > $OUT/sweep.log
timeout -k 10 400 python3 scripts/c3_tpw_sweep.py --stripes 256 --alloc 256 --slices 8,4,2 --tiles 1,2,4,8 --steps 0,64,1024,4096 --iters 10 >> $OUT/sweep.log 2> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/sweep.log'):
    d=json.loads(l); print(d['stripes'], d['ranks'], d['tiles'], d['step'], d['ms'], d['frac'])"
