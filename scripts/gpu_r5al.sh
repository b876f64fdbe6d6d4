#!/bin/bash
# Round 5, call al: the radix-2 last pass reveals a pair with both output places,
# together (ScaleIn locate / fetch / scale, branch-free; before, each row
# waited out the previous row's HBM trip): parity of the LDS reconstructs,
# then C5 repair / C4-shaped LDS timing against HEAD (labbuild/head).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5al; mkdir -p $OUT; : > $OUT/time.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rec_big.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_bsdec.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in head:$PWD/labbuild/head/librs_mi355x.so fp:$PWD/labbuild/fp/librs_mi355x.so new:$PWD/reedsolomon16_amd/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 200 python3 scripts/time_ops.py --configs C5rb8,C5r --iters 10 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/time.log'):
    d=json.loads(l); print(d['tag'], d['config'], d['us'])"
