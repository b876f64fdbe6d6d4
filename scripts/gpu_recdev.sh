#!/bin/bash
# Device reconstruct fast path: its tests, the GPU suite, then C4 wall time per
# call (caller stream, back to back) next to the kernel time (rocprofv3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/recdev
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "async_ring or reconstruct" -x -q --timeout 120 --timeout-method thread > gpurun_out/recdev/pytest_rec.log 2>&1
rc=$?; tail -3 gpurun_out/recdev/pytest_rec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/recdev/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/recdev/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/recdev/trace -o run -- python3 scripts/time_ops.py --configs C4,C4e1,C4e8,C5,C5x8,C3 --iters 50 > gpurun_out/recdev/times.jsonl 2> gpurun_out/recdev/trace.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/recdev/trace.err; exit $rc; }
cat gpurun_out/recdev/times.jsonl
cut -c1-150 gpurun_out/recdev/trace/run_kernel_stats.csv | head -8
