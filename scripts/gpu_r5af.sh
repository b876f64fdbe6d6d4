#!/bin/bash
# Round 5, call af: SQ counters of the C5 repair x 8 with packed LDS units
# (and C5 x 32 beside it), one rocprofv3 --pmc pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5af; rm -rf $OUT; mkdir -p $OUT
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o run -- python3 scripts/time_ops.py --configs C5b32,C5rb8 --iters 5 > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
(timeout -k 5 30 rocm-smi --showmemorypartition --showcomputepartition --showclocks > $OUT/smi.txt 2>&1 || true)
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt; grep -E "k_rec|k_enc" $OUT/summary.txt
