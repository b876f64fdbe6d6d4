#!/bin/bash
# Round 4: per-phase cost of the C4 decoder (k_rec_bs256): HIP-event time and
# SQ_INSTS_VALU of each RS_DEC_ABL lab build (scripts/ablate_dec.sh; steps
# left out, results wrong) at C4 x 16.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4g; mkdir -p $OUT; : > $OUT/time.log
for d in build/ablate_dec/*/; do
  n=$(basename $d)
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -k 10 60 python3 scripts/time_ops.py --configs C4x16 --iters 20 --tag $n >> $OUT/time.log 2> $OUT/$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "time $n rc=$rc"; tail -3 $OUT/$n.err; exit $rc; }
  RS_MI355X_LIB=$PWD/$d/librs_mi355x.so timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_$n -o run -- python3 scripts/time_ops.py --configs C4x16 --iters 3 > $OUT/pmc_$n.out 2> $OUT/pmc_$n.err
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $n rc=$rc"; tail -3 $OUT/pmc_$n.err; exit $rc; }
done
grep '{' $OUT/time.log
for d in $OUT/pmc_*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_rec_bs256 ; done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
