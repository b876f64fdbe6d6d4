#!/bin/bash
# Round 6, call c: the multi-device codec's GPU tests (devices = [0,0,0,0]),
# the two-thread stream test, then a tiles-per-workgroup sweep that reaches
# one-generation (persistent) grids for the byte-range slices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6c
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_stream_suites.py -x -v --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1,2,4,8 --tiles 1,4,8,16,32,64 --iters 20 > $OUT/sweep.jsonl 2> $OUT/sweep.err
rc=$?; echo "sweep rc=$rc"; cat $OUT/sweep.jsonl; exit $rc
