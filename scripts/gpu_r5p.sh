#!/bin/bash
# Round 5, call p: C3 auto tile rule check (tiles 0 = auto vs 1 / 4) on one box,
# then the bench line's C3 leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5p; mkdir -p $OUT
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1,8,4 --tiles 0,1,4 --steps 0 --iters 20 > $OUT/sweep.log 2> $OUT/sweep.err || { tail -3 $OUT/sweep.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu --no-host --no-other > $OUT/bench.json 2> $OUT/bench.err || { tail -3 $OUT/bench.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/sweep.log'):
    d=json.loads(l); print(d['stripes'], d['ranks'], d['tiles'], d['ms'], d['frac'])
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d.get('single_stripe',{}).get('frac') if isinstance(d.get('single_stripe'),dict) else '')"
