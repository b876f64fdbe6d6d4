#!/bin/bash
# Round 4: C3 bench row-stagger sweep (rows at S + pad), two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4r; mkdir -p $OUT
for pass in 1 2; do
for pad in ${PADS:-1024 2048 3072 4608 5120 6144 7168 9216 11264}; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-other --no-single --no-unpadded --steps 50 --warmup 5 --row-pad $pad > $OUT/b_$pad.json 2> $OUT/b_$pad.err
  rc=$?; [ $rc -eq 0 ] || { echo "pad $pad rc=$rc"; tail -3 $OUT/b_$pad.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/b_$pad.json'));print('pad', $pad, d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
done
