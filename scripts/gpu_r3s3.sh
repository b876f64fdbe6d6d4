#!/bin/bash
# Round-3 (session 3) evidence: GPU suite; C4 / C5 kernel stats (rocprofv3 --stats) and HIP-event times;
# SQ and HBM counters of the C4 decode at 16 stripes (separate --pmc passes); host-resident stream timings
# (encode / verify / reconstruct, one call per block vs tickets).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3s3; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/time_ops.py --configs C4,C4x16,C5,C5b32,C5x8b32 --iters 20 --tag r3s3 > $OUT/times.txt 2>&1
rc=$?; echo "times rc=$rc"; grep '{' $OUT/times.txt; [ $rc -eq 0 ] || exit $rc
run() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o run -- "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run c4_p1 "$P1" python3 scripts/time_ops.py --configs C4x16 --iters 10
run c4_p2 "$P2" python3 scripts/time_ops.py --configs C4x16 --iters 10
run c4_fetch FETCH_SIZE python3 scripts/time_ops.py --configs C4x16 --iters 10
run c4_write WRITE_SIZE python3 scripts/time_ops.py --configs C4x16 --iters 10
for d in $OUT/c4_*/; do echo "== $d"; python3 scripts/pmc_summary.py ${d%/} k_ ; done > $OUT/pmc_summary.txt 2>&1
cat $OUT/pmc_summary.txt | head -40
timeout -k 10 300 python3 scripts/time_ops.py --configs H3s_sync,H3s_async,H3vs_sync,H3vs_async,H4s_sync,H4s_async --iters 10 --tag r3s3 > $OUT/host.txt 2>&1
rc=$?; echo "host rc=$rc"; grep '{' $OUT/host.txt; [ $rc -eq 0 ] || exit $rc
