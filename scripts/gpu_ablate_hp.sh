#!/bin/bash
# Time each library under build/ablate_hp/ with the bench workload (C3, --stripes per launch, default 128,
# plus its one-stripe figure), two passes.  No parity check: some ablations are wrong on purpose.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ablate_hp.log
for pass in 1 2; do
for d in build/ablate_hp/*/; do
  n=$(basename $d)
  [ "$n" = common ] && continue
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 python bench.py --no-cpu --no-other --no-unpadded --steps ${STEPS:-100} --warmup 10 --stripes ${STRIPES:-128} > gpurun_out/abh_${n}.json 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 gpurun_out/abh_${n}.json; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abh_${n}.json').read().strip().splitlines()[-1]); print('$n', d['roofline']['kernel_ms'], d['roofline']['frac'], 'single', d['single_stripe']['kernel_ms'], d['single_stripe']['frac'])" >> gpurun_out/ablate_hp.log
done
done
cat gpurun_out/ablate_hp.log
