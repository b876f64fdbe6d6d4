#!/bin/bash
# Round 5, call ac: is the 8-rank C3 slice's lower fraction the launch size or
# the slice shape?  Slices of 1 and 8 ranks at 256..2048 stripes per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5ac; mkdir -p $OUT
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 2048,1024,512,256 --slices 8 --tiles 0,1 --iters 10 > $OUT/s8.log 2> $OUT/s8.err || { tail -3 $OUT/s8.err; exit 1; }
timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1 --tiles 0 --iters 10 > $OUT/s1.log 2> $OUT/s1.err || { tail -3 $OUT/s1.err; exit 1; }
cat $OUT/s8.log $OUT/s1.log
