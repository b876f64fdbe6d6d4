#!/bin/bash
# Bit-sliced n = 256 reconstruct parity tests only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/bsdec; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsdec.py -x -v --timeout 120 --timeout-method thread "$@" > $OUT/pytest_bsdec.log 2>&1
rc=$?; tail -25 $OUT/pytest_bsdec.log; exit $rc
