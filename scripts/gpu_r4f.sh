#!/bin/bash
# Round 4: big-n reconstruct with 1024-thread workgroups: parity, C5-repair timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rec_big.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/recbig.log 2>&1
rc=$?; echo "recbig rc=$rc"; tail -5 $OUT/recbig.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/time_ops.py --configs C5r,C5rb8 --iters 10 > $OUT/time.log 2>&1
echo "time rc=$?"; grep '{' $OUT/time.log
