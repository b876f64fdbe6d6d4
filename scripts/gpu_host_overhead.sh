#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/host_overhead.py > gpurun_out/host_overhead.log 2>&1; rc=$?
grep '^{' gpurun_out/host_overhead.log; exit $rc
