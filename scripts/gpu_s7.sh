#!/bin/bash
# GPU suite, then host-resident (PCIe-inclusive) rates: encode, reconstruct into fresh vs caller (pinned) rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s7
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s7/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s7/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/time_ops.py --configs H3p,H4p,H4pc,H3vp,H3s_async,C4,C5 --iters 40 > gpurun_out/s7/time_ops.log 2>&1
rc=$?; echo "time rc=$rc"; grep '{' gpurun_out/s7/time_ops.log; exit $rc
