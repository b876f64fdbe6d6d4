#!/bin/bash
# Diagnostics for the fused encode kernel: stamp lab + SQ counter passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/diag
mkdir -p $OUT
if [ -x scripts/micro/encode_lab ]; then
  timeout -k 5 60 scripts/micro/encode_lab > $OUT/lab.txt 2>&1; rc=$?; echo "lab rc=$rc"; cat $OUT/lab.txt; [ $rc -eq 0 ] || exit $rc
fi
i=0
IFS='|'
for pmc in ${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU|SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM GRBM_GUI_ACTIVE}; do
  i=$((i+1))
  IFS=' '
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o run -- python3 scripts/prof_encode.py ${PROF_ARGS:---iters 10} > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  IFS='|'
done
python3 scripts/pmc_summary.py $OUT encode
exit 0
