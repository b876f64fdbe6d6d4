#!/bin/bash
# Round 4 A/B: C3 encode with lane-contiguous loads + quad transpose (new
# librs_mi355x.so) vs the block-per-lane loads (lib_base); parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bitslice.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
for v in base:reedsolomon16_amd/lib_base.so ld:reedsolomon16_amd/lib_ld.so ldst:reedsolomon16_amd/librs_mi355x.so; do
  n=${v%%:*}; lib=${v#*:}
  RS_MI355X_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu --no-other --steps 50 --warmup 5 > $OUT/bench_$n.json 2> $OUT/bench_$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $n rc=$rc"; tail -3 $OUT/bench_$n.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('$n', d['roofline']['kernel_ms'], d['roofline']['frac'], d['single_stripe'], d.get('unpadded_rows'))"
done
done
ABLIBS='base:reedsolomon16_amd/lib_base.so ld:reedsolomon16_amd/lib_ld.so ldst:reedsolomon16_amd/librs_mi355x.so' CONFIGS=C3x16,C3vx16 ITERS=20 bash scripts/gpu_ab.sh
