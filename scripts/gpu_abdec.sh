#!/bin/bash
# Same-box A/B of decoder libraries under build/ablate_dec/ (HIP events, scripts/time_ops.py), two passes;
# a library named "stamp" (RS_DEC_STAMP build) prints its per-wave segment cycles to stderr.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abdec; mkdir -p $OUT; : > $OUT/ablate.log
if [ -n "$TESTS" ]; then timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc; fi
for pass in 1 2; do
for d in build/ablate_dec/*/; do
  n=$(basename $d)
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 90 python3 scripts/time_ops.py --configs ${CONFIGS:-C4,C4x16} --iters 30 --tag $n >> $OUT/ablate.log 2> $OUT/$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
done
done
grep '{' $OUT/ablate.log
grep -A13 "stamps" $OUT/stamp.err | head -30
