#!/bin/bash
# A/B timing of library builds in one call (same box): ABLIBS="name:path ...",
# CONFIGS for scripts/time_ops.py; two alternating passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab; mkdir -p $OUT; : > $OUT/time.log
for pass in 1 2; do
for v in $ABLIBS; do
  n=${v%%:*}; lib=${v#*:}
  RS_MI355X_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/time_ops.py --configs $CONFIGS --iters ${ITERS:-20} --tag $n >> $OUT/time.log 2> $OUT/$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; tail -3 $OUT/$n.err; exit $rc; }
done
done
grep '{' $OUT/time.log
