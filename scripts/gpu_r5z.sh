#!/bin/bash
# Round 5, call z: the per-rank launch shapes of the N-GPU byte-range split on
# one GPU (bench.py --slice-of N), full rows beside them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5z; mkdir -p $OUT; : > $OUT/slices.log
for n in 1 2 4 8; do
  if [ $n -eq 1 ]; then A=""; else A="--slice-of $n"; fi
  timeout -k 10 300 python bench.py $A --no-cpu --no-host --no-other --no-single --no-unpadded --steps 100 --warmup 10 >> $OUT/slices.log 2> $OUT/s$n.err || { tail -3 $OUT/s$n.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/slices.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config']['parallelism'][:70], d['roofline']['kernel_ms'], d['roofline']['frac'], d['value'])"
