#!/bin/bash
# Round-4 C4 / C5 / C5-repair kernel evidence: rocprofv3 kernel trace of the
# time_ops shapes (averaged per launch shape by scripts/trace_by_shape.py),
# and SQ VALU counters of the C5 encode (32 stripes) and the C5 repair
# (8 stripes) in separate --pmc passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4v; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/time_ops.py --configs C4,C4x16,C5,C5b32,C5x8b32,C5r,C5rb8 --iters 20 --tag r4v > $OUT/times.txt 2>&1
rc=$?; echo "times rc=$rc"; grep '{' $OUT/times.txt; [ $rc -eq 0 ] || exit $rc
python3 scripts/trace_by_shape.py $OUT/trace > $OUT/by_shape.txt; cat $OUT/by_shape.txt
run() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
run c5_p1 "$P1" python3 scripts/time_ops.py --configs C5b32 --iters 5
run c5r_p1 "$P1" python3 scripts/time_ops.py --configs C5rb8 --iters 5
run c5_grbm GRBM_GUI_ACTIVE python3 scripts/time_ops.py --configs C5b32 --iters 5
run c5r_grbm GRBM_GUI_ACTIVE python3 scripts/time_ops.py --configs C5rb8 --iters 5
for d in $OUT/c5*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_ ; done > $OUT/pmc_summary.txt 2>&1
cat $OUT/pmc_summary.txt | head -60
