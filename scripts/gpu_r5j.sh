#!/bin/bash
# Round 5, call j: C3 tile-to-workgroup maps: tiles per workgroup x tile
# distance, on exact and oversized allocations; then the tiles-per-workgroup
# parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5j; mkdir -p $OUT; : > $OUT/sweep.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bitslice.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "256 256" "256 320" "128 128" "192 192"; do
  set -- $spec
  timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --stripes $1 --alloc $2 --slices 1 --tiles 1,2,4 --steps 0,512,2048,8192 >> $OUT/sweep.log 2> $OUT/sweep.err || { tail -5 $OUT/sweep.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/sweep.log'):
    d=json.loads(l); print(d['stripes'], d['alloc'], d['tiles'], d['step'], d['ms'], d['frac'])"
