#!/bin/bash
# Round 5, call ae: does the C3 tile map's rate depend on the size of the
# allocation the rows live in?  The same launches (8-rank slices of 256
# stripes; full rows of 128 stripes) inside buffers allocated for 1x, 2x, 4x
# and 8x the launched stripes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5ae; mkdir -p $OUT; : > $OUT/a.log
for al in 256 512 1024 2048; do
  timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 8 --tiles 0,1 --alloc $al --iters 10 >> $OUT/a.log 2> $OUT/a.err || { tail -3 $OUT/a.err; exit 1; }
done
for al in 128 256 512; do
  timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 128 --slices 1 --tiles 0,4 --alloc $al --iters 10 >> $OUT/a.log 2> $OUT/a.err || { tail -3 $OUT/a.err; exit 1; }
done
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1 --tiles 0 --alloc 256 --iters 10 >> $OUT/a.log 2> $OUT/a.err || { tail -3 $OUT/a.err; exit 1; }
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1 --tiles 0 --alloc 512 --iters 10 >> $OUT/a.log 2> $OUT/a.err || { tail -3 $OUT/a.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/a.log'):
    d=json.loads(l); print(d['stripes'], d['ranks'], d['tiles'], d['alloc'], d['ms'], d['frac'])"
