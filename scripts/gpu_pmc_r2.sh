#!/bin/bash
# Round-2 counter passes (one rocprofv3 --pmc run per counter group, each under
# its own time limit): C3 bench (k_encode_hp), C4 reconstruct and C5 encode
# (scripts/time_ops.py).  Summaries: python scripts/pmc_summary.py <dir> <kernel>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc2
rm -rf $OUT; mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
for W in C3; do
  run ${W}_p1 "$P1" python3 bench.py --no-cpu --no-single --no-unpadded --stripes 32 --steps 20 --warmup 3
  run ${W}_p2 "$P2" python3 bench.py --no-cpu --no-single --no-unpadded --stripes 32 --steps 20 --warmup 3
  run ${W}_fetch FETCH_SIZE python3 bench.py --no-cpu --no-single --no-unpadded --stripes 32 --steps 20 --warmup 3
  run ${W}_write WRITE_SIZE python3 bench.py --no-cpu --no-single --no-unpadded --stripes 32 --steps 20 --warmup 3
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lds_trace -o run -- python3 scripts/time_ops.py --configs C4,C4e1,C5,C5x8 --iters 30 > $OUT/lds_trace.out 2> $OUT/lds_trace.err
rc=$?; echo "lds trace rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/lds_trace.err; exit $rc; }
for W in C4 C5 C5x8; do
  run ${W}_p1 "$P1" python3 scripts/time_ops.py --configs $W --iters 20
  run ${W}_p2 "$P2" python3 scripts/time_ops.py --configs $W --iters 20
  run ${W}_fetch FETCH_SIZE python3 scripts/time_ops.py --configs $W --iters 20
  run ${W}_write WRITE_SIZE python3 scripts/time_ops.py --configs $W --iters 20
done
for d in $OUT/*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_ ; done > $OUT/summary.txt 2>&1
cat $OUT/summary.txt | head -80
