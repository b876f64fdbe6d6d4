#!/bin/bash
# RS_NULL_STREAM: GPU suite, per-call host vs GPU time, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/host_overhead.py > gpurun_out/host_overhead.log 2>&1 || { tail -5 gpurun_out/host_overhead.log; exit 1; }
grep '^{' gpurun_out/host_overhead.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_s0.log 2>&1 || { tail -5 gpurun_out/bench_s0.log; exit 1; }
tail -1 gpurun_out/bench_s0.log
timeout -k 10 200 python scripts/time_ops.py --configs C4,C4e1,C5,C5x8 --iters 50 > gpurun_out/time_ops_s0.jsonl 2>&1; rc=$?
cat gpurun_out/time_ops_s0.jsonl; exit $rc
