#!/bin/bash
# Bench at the new default batch and a stripe sweep of the full-row and 8-rank-slice C3 launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench64.log 2>&1 || { tail -5 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log
: > gpurun_out/sweep2.log
for B in 16 32 64 96; do
  timeout -k 10 200 python scripts/time_geoms.py --stripes $B 128:32 >> gpurun_out/sweep2.log 2>&1 || exit 1
done
for B in 64 128 256; do
  timeout -k 10 200 python scripts/time_geoms.py --stripes $B --shard 131072 128:32 >> gpurun_out/sweep2.log 2>&1 || exit 1
done
grep '^{' gpurun_out/sweep2.log
