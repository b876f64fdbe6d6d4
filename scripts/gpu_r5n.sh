#!/bin/bash
# Round 5, call n: the reference stream suites through the engine, then the
# C3 per-rank slice sweep (tiles per workgroup x tile distance).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream_suites.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r5m.sh
