#!/bin/bash
# GPU suite on the register-accumulator LDS encode, then C5 A/B of build/ablate/*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s6/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s6/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS=C4,C4 ./scripts/gpu_ablate_rec.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
CONFIGS=C4,C4e1 ./scripts/gpu_ablate_rec.sh; exit $?
