#!/bin/bash
# Round 4: the LDS-resident reconstruct for n = 512..2048 (parity first), its
# C5-repair timing, then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rec_big.py -x -q --timeout 120 --timeout-method thread > $OUT/recbig.log 2>&1
rc=$?; echo "recbig rc=$rc"; tail -15 $OUT/recbig.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/time_ops.py --configs C5r,C5rb8,C4x16 --iters 10 > $OUT/time.log 2>&1
echo "time rc=$?"; grep '{' $OUT/time.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
