#!/bin/bash
# Round 5, call l: C4 decoder with the reveal rolled through LDS (71 KB of
# code): parity tests, then timing against round 4 (112 KB) and the single
# phase-1 call site (81 KB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5l; mkdir -p $OUT; : > $OUT/time.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsdec.py tests/test_gpu_golden.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in r4:$PWD/labbuild/old_dec/librs_mi355x.so k81:$PWD/labbuild/dec81/librs_mi355x.so k71:$PWD/reedsolomon16_amd/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C4x16,C4,C4e1,C4e4 --iters 20 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/time.log'):
    d=json.loads(l); print(d['tag'], d['config'], d['us'])"
