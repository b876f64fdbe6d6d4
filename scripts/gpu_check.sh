#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first crash
# (abort / segfault / timeout); plain test failures (exit 1) still let the
# remaining steps run so their output can be read.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 ${PYTEST_TIMEOUT:-420} python -m pytest tests -m gpu -q -ra ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok_or_testfail $rc || exit $rc

timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
ok_or_testfail $rc || exit $rc

timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
