#!/bin/bash
# Parity tests (fast subset unless FULL=1) + timing of the BASELINE configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/time_ops.py --configs ${CFGS:-C2,C3,C3v,C4,C5,C5x8,H3,H3p,H4p,H3vp} --iters 50 > gpurun_out/time_ops.log 2>&1
rc=$?; echo "time rc=$rc"; grep '{' gpurun_out/time_ops.log
exit $rc
