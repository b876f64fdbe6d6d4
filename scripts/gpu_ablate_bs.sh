#!/bin/bash
# Time each bit-sliced ablation library (build/ablate_bs/<name>/, from
# scripts/ablate_bs.sh) with the bench workload: C3, 16 stripes per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ablate_bs.log
for d in build/ablate_bs/*/; do
  n=$(basename $d)
  [ "$n" = common ] && continue
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 180 python -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_${n}_pytest.log 2>&1
  rc=$?; echo "$n pytest rc=$rc $(tail -1 gpurun_out/ab_${n}_pytest.log)" >> gpurun_out/ablate_bs.log; [ $rc -eq 0 ] || { cat gpurun_out/ablate_bs.log; tail -30 gpurun_out/ab_${n}_pytest.log; exit $rc; }
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-100} --warmup 10 > gpurun_out/ab_$n.json 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "fail $n rc=$rc"; tail -5 gpurun_out/ab_$n.json; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/ablate_bs.log
done
cat gpurun_out/ablate_bs.log
