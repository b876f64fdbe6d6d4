#!/bin/bash
# Few-erasure repair: LDS reconstruct kernel time with and without FFT pruning.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/prune_times.jsonl
for np_ in 0 1; do
  RS_NO_PRUNE=$np_ timeout -k 10 120 python scripts/time_ops.py --configs C4,C4e1,C4e2,C4e4,C4e8 --iters 50 >> gpurun_out/prune_times.jsonl 2>gpurun_out/prune_err.log || { tail -5 gpurun_out/prune_err.log; exit 1; }
done
cat gpurun_out/prune_times.jsonl
timeout -k 10 200 python scripts/time_ops.py --configs H3s_sync,H3s_async,H3p --iters 10 > gpurun_out/stream_times.jsonl 2>gpurun_out/stream_err.log || { tail -5 gpurun_out/stream_err.log; exit 1; }
cat gpurun_out/stream_times.jsonl
