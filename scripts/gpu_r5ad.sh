#!/bin/bash
# Round 5, call ad: single-tile tail for the four-tiles-per-workgroup C3
# encode (BsArgs head_tiles / head_wgs, knob hp_tail): parity, then the
# tiles x tail sweep on full rows and on the per-rank slices of 2/4/8 ranks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5ad; mkdir -p $OUT
true

for pass in 1 2; do
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256,128,64 --slices 1 --tiles 0,1,4 --tails=-1,0,512,2048 --iters 10 >> $OUT/full.log 2> $OUT/full.err || { tail -3 $OUT/full.err; exit 1; }
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 2,4,8 --tiles 0,1 --tails=-1,0,512,2048 --iters 10 >> $OUT/slices.log 2> $OUT/slices.err || { tail -3 $OUT/slices.err; exit 1; }
done
python3 -c "
import json
for f in ('full','slices'):
    for l in open('$OUT/'+f+'.log'):
        d=json.loads(l); print(d['stripes'], d['ranks'], d['tiles'], d['tail'], d['ms'], d['frac'])"
