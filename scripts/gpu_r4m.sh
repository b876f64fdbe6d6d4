#!/bin/bash
# Round 4: SQ counters of the big-n LDS reconstruct (C5 repair x 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4m; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for P in P1 P2; do
  timeout -s KILL 120 rocprofv3 --pmc ${!P} --output-format csv -d $OUT/$P -o run -- python3 scripts/time_ops.py --configs C5rb8 --iters 2 > $OUT/$P.out 2> $OUT/$P.err
  rc=$?; echo "$P rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$P.err; exit $rc; }
done
for d in $OUT/P*/; do python3 scripts/pmc_summary.py ${d%/} k_rec ; done
