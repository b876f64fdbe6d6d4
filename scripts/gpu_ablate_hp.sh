#!/bin/bash
# Time each library under build/ablate_hp/ with the bench workload (C3, 16
# stripes per launch, and 1 stripe).  No parity check: ablations are wrong on purpose.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ablate_hp.log
for d in build/ablate_hp/*/; do
  n=$(basename $d)
  [ "$n" = common ] && continue
  for B in 16 1; do
    RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-100} --warmup 10 --stripes $B > gpurun_out/abh_${n}_$B.json 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 gpurun_out/abh_${n}_$B.json; exit $rc; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abh_${n}_$B.json').read().strip().splitlines()[-1]); print('$n', 'stripes=$B', d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/ablate_hp.log
  done
done
cat gpurun_out/ablate_hp.log
