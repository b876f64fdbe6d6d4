#!/bin/bash
# Round 4: stream6 lab (engine-like occupancy); big-n reconstruct XCD tile
# pairing A/B (lib_old = identity map), parity, FETCH_SIZE of the new map.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 200 scripts/micro/stream6_lab > $OUT/stream6.txt 2>&1
rc=$?; echo "lab rc=$rc"; grep -A60 "pass 1" $OUT/stream6.txt | grep -i "LDS\|512B bs256 \|2048B bs256 "; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_rec_big.py -x -q --timeout 120 --timeout-method thread > $OUT/recbig.log 2>&1
rc=$?; echo "recbig rc=$rc"; tail -2 $OUT/recbig.log; [ $rc -eq 0 ] || exit $rc
ABLIBS='old:reedsolomon16_amd/lib_old.so new:reedsolomon16_amd/librs_mi355x.so' CONFIGS=C5r,C5rb8 ITERS=5 bash scripts/gpu_ab.sh || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_f -o run -- python3 scripts/time_ops.py --configs C5rb8 --iters 2 > $OUT/pmc_f.out 2> $OUT/pmc_f.err
echo "pmc rc=$?"; python3 scripts/pmc_summary.py $OUT/pmc_f k_rec
