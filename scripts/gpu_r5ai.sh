#!/bin/bash
# Round 5, call ai: the C3 tile map on unpadded rows (rows exactly 1 MiB
# apart, the reference's AllocAligned layout): tiles per workgroup x tile
# distance, against the padded layout on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5ai; mkdir -p $OUT; : > $OUT/a.log
timeout -k 10 400 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1 --tiles 1,2,4,8 --steps 0,64,512,4096 --pad 0 --iters 10 >> $OUT/a.log 2> $OUT/a.err || { tail -3 $OUT/a.err; exit 1; }
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1 --tiles 1,4 --pad 3584 --iters 10 >> $OUT/a.log 2> $OUT/a.err || { tail -3 $OUT/a.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/a.log'):
    d=json.loads(l); print(d['pad'], d['tiles'], d['step'], d['ms'], d['frac'])"
