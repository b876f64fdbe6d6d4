#!/bin/bash
# Round 4: same-box calibration table (copy / read / write labs, C3-pattern
# labs, the engine's C3 launch), and HBM traffic of the big-n LDS reconstruct
# at the C5 repair geometry (separate FETCH_SIZE / WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4h; mkdir -p $OUT
timeout -k 10 200 scripts/micro/stream5_lab > $OUT/stream5.txt 2>&1
rc=$?; echo "stream5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 scripts/micro/stream6_lab > $OUT/stream6.txt 2>&1
rc=$?; echo "stream6 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python3 scripts/time_ops.py --configs C5rb8 --iters 2 > $OUT/pmc_$c.out 2> $OUT/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/pmc_$c.err; exit $rc; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/time_ops.py --configs C5rb8 --iters 5 > $OUT/trace.out 2> $OUT/trace.err
echo "trace rc=$?"
for d in $OUT/pmc_*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_rec ; done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt; grep '{' $OUT/pmc_FETCH_SIZE.out
find $OUT/trace -name "*kernel_stats.csv" -exec head -5 {} \;
