#!/bin/bash
# Round 5, call c: C4 A/B -- product decoder vs a lab build whose phase-1 /
# phase-3 networks all use unit 0's (wrong results, 65 KB instead of 112 KB of
# code): how much the instruction cache costs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5c; mkdir -p $OUT; : > $OUT/time.log
for pass in 1 2; do
  for v in prod:$PWD/reedsolomon16_amd/librs_mi355x.so small:$PWD/labbuild/dec_small/librs_mi355x.so small5:$PWD/labbuild/dec_small5/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C4x16,C4 --iters 20 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
cat $OUT/time.log
