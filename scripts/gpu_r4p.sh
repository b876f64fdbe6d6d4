#!/bin/bash
# Round 4 A/B: C5 encode with the chunk IFFT in subfield coordinates from its
# first subfield pass on (new) vs full-field chunk IFFTs (lib_base); parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4p; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
ABLIBS='base:reedsolomon16_amd/lib_base.so new:reedsolomon16_amd/librs_mi355x.so' CONFIGS=C5,C5b32,C5x8b32,C5vb32 ITERS=10 bash scripts/gpu_ab.sh
