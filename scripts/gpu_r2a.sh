#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py > gpurun_out/bench_c3.log 2>&1 || { tail -5 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log
timeout -k 10 200 python bench.py --workload C5 --no-cpu --steps 50 > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log
timeout -k 10 60 ./scripts/micro/stream2_lab > gpurun_out/stream2_lab.log 2>&1; rc=$?
cat gpurun_out/stream2_lab.log; exit $rc
