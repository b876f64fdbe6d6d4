#!/bin/bash
# Round 4: C3-pattern small-tile lab; SQ / instruction-cache counters of the
# m = 256 encode kernels (bit-sliced k_enc_bs256 vs the LDS kernel, RS_BS=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4c; mkdir -p $OUT
timeout -k 10 200 scripts/micro/stream6_lab > $OUT/stream6.txt 2>&1
rc=$?; echo "lab rc=$rc"; cat $OUT/stream6.txt; [ $rc -eq 0 ] || exit $rc
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_WAIT_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
run() {  # name, counters, env, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
run bs_p1 "$P1" python3 scripts/time_ops.py --configs C5b32 --iters 5
run bs_p2 "$P2" python3 scripts/time_ops.py --configs C5b32 --iters 5
export RS_BS=0
run lds_p1 "$P1" python3 scripts/time_ops.py --configs C5b32 --iters 5
run lds_p2 "$P2" python3 scripts/time_ops.py --configs C5b32 --iters 5
unset RS_BS
for d in $OUT/*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_ ; done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
