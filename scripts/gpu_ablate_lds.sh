#!/bin/bash
# Time C4 / C5 (LDS-resident kernels) for each library under build/ablate/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ablate_lds.log
for d in build/ablate/*/; do
  n=$(basename $d); [ "$n" = common ] && continue
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 python scripts/time_ops.py --configs C4,C5,C5x8 --iters 30 --tag $n >> gpurun_out/ablate_lds.log 2>gpurun_out/ablate_lds_err.log || { tail -5 gpurun_out/ablate_lds_err.log; exit 1; }
done
cat gpurun_out/ablate_lds.log
