#!/bin/bash
# Round 4: new bit-sliced m = 256 encode parity first, then the full GPU suite,
# the bench line and the copy-calibration lab.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bs256.py -x -q --timeout 120 --timeout-method thread > $OUT/bs256.log 2>&1
rc=$?; echo "bs256 rc=$rc"; tail -5 $OUT/bs256.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python scripts/time_ops.py --configs C5,C5b32,C5x8b32,C5vb32,C5r,C5rb8 --iters 10 > $OUT/time_c5.log 2>&1
echo "time rc=$?"; grep '{' $OUT/time_c5.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 scripts/micro/stream5_lab > $OUT/stream5.txt 2>&1
echo "lab rc=$?"
