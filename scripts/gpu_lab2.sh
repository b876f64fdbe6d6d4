#!/bin/bash
# Round-2 calibration: the current C3 bench + issue rates of the swap/XOR instructions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --steps 50 --warmup 10 > gpurun_out/bench16.log 2>&1 || exit $?
tail -1 gpurun_out/bench16.log
timeout -k 10 200 python bench.py --no-cpu --steps 200 --warmup 20 --stripes 1 > gpurun_out/bench1.log 2>&1 || exit $?
tail -1 gpurun_out/bench1.log
timeout -k 10 60 ./scripts/micro/rate2_lab > gpurun_out/rate2_lab.log 2>&1 || { cat gpurun_out/rate2_lab.log; exit 1; }
cat gpurun_out/rate2_lab.log
