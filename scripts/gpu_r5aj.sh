#!/bin/bash
# Round 5, call aj: lab bound (wrong results) of the C5 repair's lane-varying
# twiddle tables, one pass at a time: labbuild/uD makes the tables of the
# n = 2048 passes at distance D wave-uniform (readfirstlane of the group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5aj; mkdir -p $OUT; : > $OUT/time.log
for pass in 1 2; do
  for v in prod:$PWD/reedsolomon16_amd/librs_mi355x.so u1:$PWD/labbuild/u1/librs_mi355x.so u2:$PWD/labbuild/u2/librs_mi355x.so u4:$PWD/labbuild/u4/librs_mi355x.so u8:$PWD/labbuild/u8/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 200 python3 scripts/time_ops.py --configs C5rb8 --iters 10 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/time.log'):
    d=json.loads(l); print(d['tag'], d['config'], d['us'])"
