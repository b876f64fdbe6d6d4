#!/bin/bash
# 16-row-unit bit-sliced decode (k_rec_bs256): reconstruct parity tests, then HIP-event timings and
# rocprofv3 kernel stats of C4 (one stripe, 16 stripes per launch, few erasures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/bsdec2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bsdec.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "reconstruct or C4 or c4 or recon" > $OUT/pytest_par.log 2>&1
rc=$?; tail -3 $OUT/pytest_par.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/time_ops.py --configs C4,C4x16,C4e1,C4e8 --iters 20 --tag u16 > $OUT/time.txt 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/time.txt; exit $rc; }
grep '{' $OUT/time.txt
grep -v distribution $OUT/trace/run_kernel_stats.csv | head -4
