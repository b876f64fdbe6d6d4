#!/bin/bash
# SQ counters of the bit-sliced n = 256 reconstruct (k_rec_bs256) at C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_bsdec
rm -rf $OUT; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P3="SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_IFETCH"
run() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
W=${1:-C4}
run ${W}_p1 "$P1" python3 scripts/time_ops.py --configs $W --iters 20
run ${W}_p2 "$P2" python3 scripts/time_ops.py --configs $W --iters 20
run ${W}_p3 "$P3" python3 scripts/time_ops.py --configs $W --iters 20
for d in $OUT/*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_ ; done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
