#!/bin/bash
# Fused first/last LDS passes: GPU suite first, then C4 / C5 kernel times of
# the libraries under build/ablate/ (base = this tree, old = before the change).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS=C4,C4e1,C5,C5x8 ./scripts/gpu_ablate_rec.sh
