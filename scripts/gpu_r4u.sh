#!/bin/bash
# C3 ablation A/B (scripts/ablate_hp.sh builds): bench.py's launch (128
# stripes, 3.5 KiB stagger) per lab library, two alternating passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4u; mkdir -p $OUT; : > $OUT/ab.jsonl
for pass in 1 2; do
  for n in ${NAMES:-base nonet nonet_notr memonly}; do
    RS_MI355X_LIB=$PWD/build/ablate_hp/$n/librs_mi355x.so timeout -k 10 120 python3 bench.py --stripes 128 --steps 60 --warmup 10 --no-cpu --no-single --no-unpadded --no-other > $OUT/one.json 2> $OUT/$n.err
    rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; tail -3 $OUT/$n.err; exit $rc; }
    python3 -c "
import json;d=json.loads(open('$OUT/one.json').read().strip().splitlines()[-1])
print(json.dumps({'pass':$pass,'lib':'$n','kernel_ms':d['roofline']['kernel_ms'],'frac':d['roofline']['frac']}))" | tee -a $OUT/ab.jsonl
  done
done
