#!/bin/bash
# Round 5, call e: how much the lane-varying twiddle tables of the LDS
# kernels' dist < 16 passes cost -- product vs a lab build that gives every
# lane the wave's first group (scalar table loads; wrong results).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5e; mkdir -p $OUT; : > $OUT/time.log
for pass in 1 2; do
  for v in prod:$PWD/reedsolomon16_amd/librs_mi355x.so unif:$PWD/labbuild/uniform_tw/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C5b32,C5rb8,C5 --iters 5 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/time.log'):
    d=json.loads(l); print(d['tag'], d['config'], d['us'])"
