#!/bin/bash
# Round 4 A/B: (1) big-n reconstruct, the two 64-byte tiles of a line on one
# XCD (lib_base) vs identity map (lib_nopair); (2) C3 encode, four 512-byte
# pieces per tile (librs_mi355x.so) vs one 2 KB run (lib_base); parity of the new lib.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4k; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bitslice.py tests/test_gpu_rec_big.py -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $OUT/parity.log; [ $rc -eq 0 ] || exit $rc
ABLIBS='nopair:reedsolomon16_amd/lib_nopair.so pair:reedsolomon16_amd/lib_base.so' CONFIGS=C5r,C5rb8 ITERS=5 bash scripts/gpu_ab.sh || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_f -o run -- python3 scripts/time_ops.py --configs C5rb8 --iters 2 > $OUT/pmc_f.out 2> $OUT/pmc_f.err
echo "pmc rc=$?"; python3 scripts/pmc_summary.py $OUT/pmc_f k_rec
for pass in 1 2; do
for v in base:reedsolomon16_amd/lib_base.so pieces:reedsolomon16_amd/librs_mi355x.so; do
  n=${v%%:*}; lib=${v#*:}
  RS_MI355X_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu --no-other --steps 50 --warmup 5 > $OUT/bench_$n.json 2> $OUT/bench_$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $n rc=$rc"; tail -3 $OUT/bench_$n.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$n.json'));print('$n', d['roofline']['kernel_ms'], d['roofline']['frac'], d['single_stripe'], d.get('unpadded_rows'))"
done
done
