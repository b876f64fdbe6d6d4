#!/bin/bash
# Generic bit-sliced encode: its parity tests first, then the whole GPU suite,
# the C3 bench and per-geometry timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bitslice.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gen_bs.log 2>&1
rc=$?; tail -4 gpurun_out/gen_bs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_c3.log 2>&1 || { tail -5 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
timeout -k 10 200 python scripts/time_geoms.py 128:32 130:32 192:32 100:17 32:32 64:16 192:16 16:16 20:10 > gpurun_out/gen_geoms.log 2>&1; rc=$?
cat gpurun_out/gen_geoms.log; exit $rc
