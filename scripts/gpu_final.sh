#!/bin/bash
# Round evidence: GPU suite, smoke, bench, kernel trace, FETCH/WRITE passes
# (gpu_round.sh), then the SQ / traffic counter passes for C3, C4, C5 and the
# 8-rank C5 slice with a kernel trace of the LDS kernels (gpu_pmc_r2.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
./scripts/gpu_round.sh || exit $?
./scripts/gpu_pmc_r2.sh
