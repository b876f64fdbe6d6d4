#!/bin/bash
# Round 5, call s: SQ / SQC counters of the final kernels (C3 x 16, C4 x 16,
# C5 x 32, C5 repair x 8), one rocprofv3 --pmc pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5s; rm -rf $OUT; mkdir -p $OUT
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o run -- python3 scripts/time_ops.py --configs C3x16,C4x16,C5b32,C5rb8 --iters 5 > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt; grep -E "k_rec|k_enc" $OUT/summary.txt
