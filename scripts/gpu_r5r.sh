#!/bin/bash
# Round 5, call r: C4 decoder schedule variants (scripts/lab_dec_variants.py):
# parity of each lab build on the bit-sliced decoder tests, then same-box timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5r; mkdir -p $OUT; : > $OUT/time.log
V="base bar_scale bar_load late_prio p3simd bar_scale_p3simd bar_scale_late_prio"
for n in $V; do
  RS_MI355X_LIB=$PWD/labbuild/$n/librs_mi355x.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsdec.py > $OUT/pytest_$n.log 2>&1
  rc=$?; echo "pytest $n rc=$rc $(tail -1 $OUT/pytest_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for pass in 1 2; do
  for n in $V; do
    RS_MI355X_LIB=$PWD/labbuild/$n/librs_mi355x.so timeout -k 10 120 python3 scripts/time_ops.py --configs C4x16,C4,C4e1 --iters 20 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json,collections
r=collections.defaultdict(list)
for l in open('$OUT/time.log'):
    d=json.loads(l); r[(d['tag'],d['config'])].append(d['us'])
for k,v in r.items(): print(k[0], k[1], v)"
