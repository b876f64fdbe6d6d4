#!/bin/bash
# Round 5, call u: zero-copy host reconstruct -- parity (new test + the host
# pipeline tests), then the host-resident rates with zero copy off / on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stream.py -k "host or zero_copy or async or capacity or reconstruct" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/host_zc_ab.py > $OUT/ab.log 2> $OUT/ab.err; rc=$?; cat $OUT/ab.log; [ $rc -eq 0 ] || { tail -5 $OUT/ab.err; exit $rc; }
