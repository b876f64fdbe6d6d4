#!/bin/bash
# Wave-local IFFT passes of the n > 256 reconstruct: parity (big-n tests,
# reconstruct parity, golden) then C5-repair timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4y; mkdir -p $OUT; : > $OUT/time.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rec_big.py tests/test_gpu_golden.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in ${LIBS:-new:$PWD/reedsolomon16_amd/librs_mi355x.so}; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C5r,C5rb8 --iters 10 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
grep '{' $OUT/time.log
