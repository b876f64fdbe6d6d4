#!/bin/bash
# Session check: GPU suite, C4/C5 timings, row-pad layout experiment, stream lab, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/s3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/time_ops.py --configs C4,C4,C5,C5x8,C3x16 --iters 50 > $OUT/time_ops.log 2>&1
rc=$?; echo "time rc=$rc"; cat $OUT/time_ops.log | grep '{'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/time_pad.py --pads 0,256,2048,4096,8192,65536,0 > $OUT/time_pad.log 2>&1
rc=$?; echo "pad rc=$rc"; cat $OUT/time_pad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./scripts/micro/stream2_lab > $OUT/stream2.log 2>&1
rc=$?; echo "lab rc=$rc"; cat $OUT/stream2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; exit $rc
