#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in build/ablate/*/; do
  [ "$(basename $d)" = common ] && continue
  n=$(basename $d)
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 python scripts/time_ops.py --configs ${CFGS:-C3} --tag $n >> gpurun_out/ablate.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; exit $rc; }
done
cat gpurun_out/ablate.log
