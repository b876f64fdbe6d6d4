#!/bin/bash
# LDS-resident kernel change: GPU parity first, then the ablation timing runner.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CONFIGS=${CONFIGS:-C4,C5,C5x8} ./scripts/gpu_ablate_rec.sh
timeout -k 10 200 python scripts/time_geoms.py --stripes 16 128:32 > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 200 python scripts/time_geoms.py --stripes 32 128:32 >> gpurun_out/sweep.log 2>&1 && \
timeout -k 10 200 python scripts/time_geoms.py --stripes 16 --shard 131072 128:32 >> gpurun_out/sweep.log 2>&1 && \
timeout -k 10 200 python scripts/time_geoms.py --stripes 32 --shard 131072 128:32 >> gpurun_out/sweep.log 2>&1 && \
timeout -k 10 200 python scripts/time_geoms.py --stripes 64 --shard 131072 128:32 >> gpurun_out/sweep.log 2>&1; rc=$?
grep '^{' gpurun_out/sweep.log; exit $rc
