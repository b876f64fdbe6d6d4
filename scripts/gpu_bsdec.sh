#!/bin/bash
# Bit-sliced n = 256 reconstruct: parity tests, then C4 timings against the LDS kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/bsdec; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bsdec.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_bsdec.log 2>&1
rc=$?; tail -15 $OUT/pytest_bsdec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/time_ops.py --configs C4,C4x16 --iters 30 --tag bs > $OUT/time_bs.txt 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/time_bs.txt; exit $rc; }
RS_NO_BS_DEC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_lds -o run -- python3 scripts/time_ops.py --configs C4,C4x16 --iters 30 --tag lds > $OUT/time_lds.txt 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/time_lds.txt; exit $rc; }
grep '{' $OUT/time_bs.txt $OUT/time_lds.txt
for f in $OUT/trace/*/*kernel_stats.csv $OUT/trace_lds/*/*kernel_stats.csv; do echo "== $f"; cut -d, -f1-8 $f | head -6; done
