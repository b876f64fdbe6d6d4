#!/bin/bash
# Round 5, call t: host <-> device row copies for the host-resident reconstruct
# (scripts/micro/zc_lab.hip): per-row hipMemcpyAsync vs zero-copy gather /
# scatter kernels over pinned host rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5t; mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/micro/zc_lab.hip -o /tmp/zc_lab > $OUT/build.log 2>&1 || { tail -5 $OUT/build.log; exit 1; }
timeout -k 10 180 /tmp/zc_lab > $OUT/zc.log 2>&1; rc=$?; cat $OUT/zc.log; exit $rc
