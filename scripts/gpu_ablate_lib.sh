#!/bin/bash
# Time each library under build/ablate/ (HIP events, scripts/time_ops.py CONFIGS), two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ablib; mkdir -p $OUT; : > $OUT/ablate.log
for pass in 1 2; do
for d in build/ablate/*/; do
  n=$(basename $d); [ "$n" = common ] && continue
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 python3 scripts/time_ops.py --configs ${CONFIGS:-C5,C5b32,C5x8b32} --iters 10 --tag $n >> $OUT/ablate.log 2> $OUT/$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 $OUT/$n.err; exit $rc; }
done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/ablib/ablate.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["tag"], d["config"], d["us"], d["frac"])
PY
