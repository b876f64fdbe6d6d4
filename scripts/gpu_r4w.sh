#!/bin/bash
# k_enc_lds occupancy A/B (scripts/ablate_enc.sh): the product library (128-byte
# tiles) against 64-byte tiles at N workgroups per CU, C5 shapes, two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4w; mkdir -p $OUT; : > $OUT/time.log
for pass in 1 2; do
  RS_MI355X_LIB=$PWD/reedsolomon16_amd/librs_mi355x.so timeout -k 10 120 python3 scripts/time_ops.py --configs C5b32,C5x8b32 --iters 10 --tag wide >> $OUT/time.log 2> $OUT/wide.err || { tail -3 $OUT/wide.err; exit 1; }
  for n in ${WGS:-4 5 6 8}; do
    RS_UNIT_WIDTH=narrow RS_MI355X_LIB=$PWD/build/ablate_enc/w$n/librs_mi355x.so timeout -k 10 120 python3 scripts/time_ops.py --configs C5b32,C5x8b32 --iters 10 --tag narrow_w$n >> $OUT/time.log 2> $OUT/w$n.err || { tail -3 $OUT/w$n.err; exit 1; }
  done
done
grep '{' $OUT/time.log
