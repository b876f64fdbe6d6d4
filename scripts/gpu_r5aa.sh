#!/bin/bash
# Round 5, call aa: C4 decoder putting phase-1 units behind per-unit
# phase-3-done tokens (no image-free barrier): parity, then C4 timing
# against the previous build (labbuild/base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5aa; mkdir -p $OUT; : > $OUT/time.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsdec.py tests/test_gpu_golden.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in base:$PWD/labbuild/base/librs_mi355x.so tok:$PWD/reedsolomon16_amd/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C4x16,C4,C4e1,C4e4 --iters 20 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('$OUT/time.log'):
    d=json.loads(l); r[(d['tag'],d['config'])].append(d['us'])
for k,v in sorted(r.items(), key=lambda kv: (kv[0][1], kv[0][0])): print(k[0], k[1], v)"
