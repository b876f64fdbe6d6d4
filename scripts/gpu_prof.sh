#!/bin/bash
# Profile the headline encode: kernel trace stats + PMC passes (separate runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="${PROF_ARGS:---iters 20}"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/prof_encode.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for pmc in ${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "FETCH_SIZE" "WRITE_SIZE"}; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- python3 scripts/prof_encode.py $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($pmc) rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
exit 0
