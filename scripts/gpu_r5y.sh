#!/bin/bash
# Round 5, call y: the stream mirror with a block's readers / writers on 8
# threads -- GPU stream tests, then the host-resident rates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5y; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py tests/test_gpu_stream_suites.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/host_zc_ab.py > $OUT/ab.log 2> $OUT/ab.err; rc=$?; cat $OUT/ab.log; [ $rc -eq 0 ] || { tail -5 $OUT/ab.err; exit $rc; }
