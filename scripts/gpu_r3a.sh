#!/bin/bash
# Round 3, first GPU call: GPU suite after the round-2 cleanup, the bench line,
# and the C3 memory-pattern lab (stream3_lab).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./scripts/micro/stream3_lab > $OUT/stream3.txt 2>&1
rc=$?; echo "lab rc=$rc"; cat $OUT/stream3.txt
exit $rc
