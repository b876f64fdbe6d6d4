#!/bin/bash
# Round 4 A/B: big-n reconstruct with its subfield passes (new) vs full field (lib_base); parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4q; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_rec_big.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
ABLIBS='base:reedsolomon16_amd/lib_base.so new:reedsolomon16_amd/librs_mi355x.so' CONFIGS=C5r,C5rb8 ITERS=5 bash scripts/gpu_ab.sh
