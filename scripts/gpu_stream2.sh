#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/micro/stream2_lab > gpurun_out/stream2_lab.log 2>&1; rc=$?
cat gpurun_out/stream2_lab.log; exit $rc
