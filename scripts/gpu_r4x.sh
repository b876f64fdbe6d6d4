#!/bin/bash
# 256-byte encode tiles (F16<8>, build/ablate_w8): parity of the m > 32 encode
# tests against the oracle through the lab library, then C5 timing A/B
# against the product library (two passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4x; mkdir -p $OUT; : > $OUT/time.log
L8=$PWD/build/ablate_w8/librs_mi355x.so
RS_MI355X_LIB=$L8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "encode or c5 or verify or subfield" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in prod:$PWD/reedsolomon16_amd/librs_mi355x.so w8:$L8; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C5,C5b32,C5x8b32,C5vb32 --iters 10 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
grep '{' $OUT/time.log
