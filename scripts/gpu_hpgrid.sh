#!/bin/bash
# A/B of the C3 launch shape: persistent grid (2 workgroups per CU) vs one tile per workgroup.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hpgrid; mkdir -p $OUT; : > $OUT/ab.txt
for r in 1 2; do
  for g in pers tiles; do
    if [ $g = pers ]; then export RS_HP_GRID=2; else unset RS_HP_GRID; fi
    timeout -k 10 120 python bench.py --no-cpu --no-unpadded --steps 30 --warmup 5 > $OUT/b_$g.json 2>>$OUT/err.txt || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/b_$g.json')); print('$g', d['roofline']['kernel_ms'], d['roofline']['frac'], d['single_stripe'])" >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
