#!/bin/bash
# Verify A/B: parity via LDS-DMA (base) vs loaded at the compare (vnodma), on encoded (passing) stripes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do for v in base vnodma; do
  RS_MI355X_LIB=$PWD/build/ablate_hp/$v/librs_mi355x.so timeout -k 10 120 python scripts/time_ops.py --configs C3vx16,C3v,C3x16 --iters 30 --tag $v > gpurun_out/vab_$v.log 2>&1 || exit $?
  grep '{' gpurun_out/vab_$v.log
done; done
