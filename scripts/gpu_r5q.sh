#!/bin/bash
# Round 5, call q: per-wave phase stamps of the C4 decoder (lab build), then
# the C3 auto tile rule check and the bench line's C3 leg (call p).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5q; mkdir -p $OUT
RS_MI355X_LIB=$PWD/labbuild/stamp/librs_mi355x.so timeout -k 10 120 python3 scripts/dec_stamp_run.py > $OUT/stamps.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.json
bash scripts/gpu_r5p.sh
