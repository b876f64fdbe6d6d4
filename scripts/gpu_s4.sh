#!/bin/bash
# GPU suite on the swizzled-LDS library, then C4/C5 A/B of build/ablate/* under
# rocprofv3, then a repeated C3 row-pad layout sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s4/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS=C4,C4e1,C5,C5x8 ./scripts/gpu_ablate_rec.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
CONFIGS=C4,C5 ./scripts/gpu_ablate_rec.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/time_pad.py --pads 0,1024,3072,0,1024,3072,0,1024,3072 --iters 40 > gpurun_out/s4/time_pad.log 2>&1
rc=$?; echo "pad rc=$rc"; cat gpurun_out/s4/time_pad.log; exit $rc
