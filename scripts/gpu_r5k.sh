#!/bin/bash
# Round 5, call k: C3 tiles per workgroup at large launches, exact allocations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5k; mkdir -p $OUT; : > $OUT/sweep.log
for st in 256 320 384 512 224; do
  timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --stripes $st --alloc $st --slices 1 --tiles 1,2,4,8 --iters 10 >> $OUT/sweep.log 2> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
done
timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --stripes 256 --alloc 256 --slices 2,4,8 --tiles 1,2,4,8 --iters 10 >> $OUT/sweep.log 2>> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/sweep.log'):
    d=json.loads(l); print(d['stripes'], d['ranks'], d['tiles'], d['ms'], d['frac'])"
