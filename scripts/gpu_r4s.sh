#!/bin/bash
# Round 4: row stagger for the per-rank byte-range slices (bench.py --slice-of N).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4s; mkdir -p $OUT
for pass in 1 2; do
for n in 2 8; do
for pad in 1536 3072 3584 4608; do
  timeout -k 10 200 python3 bench.py --slice-of $n --no-cpu --no-other --no-single --no-unpadded --steps 50 --warmup 5 --row-pad $pad > $OUT/b.json 2> $OUT/b.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 $OUT/b.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('slice', $n, 'pad', $pad, d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
done
done
