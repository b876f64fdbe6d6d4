#!/bin/bash
# Time C4 for each library under build/ablate_dec/ (HIP events, scripts/time_ops.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abdec; mkdir -p $OUT; : > $OUT/ablate.log
for pass in 1 2; do
for d in build/ablate_dec/*/; do
  n=$(basename $d)
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 60 python3 scripts/time_ops.py --configs ${CONFIGS:-C4,C4x16} --iters 30 --tag $n >> $OUT/ablate.log 2> $OUT/$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
done
done
grep '{' $OUT/ablate.log
