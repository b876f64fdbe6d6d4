#!/bin/bash
# Wide-tile m = 256 encode (k_enc_wide) vs the 128-byte-tile LDS kernel: parity tests, then HIP-event
# timings and rocprofv3 kernel stats of C5 / C5 batched / the 8-rank slice with RS_ENC_WIDE=1 and 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/wide; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "wide_encode or c5 or C5 or unit_width or batch" > $OUT/pytest_wide.log 2>&1
rc=$?; tail -3 $OUT/pytest_wide.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  export RS_ENC_WIDE=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$v -o run -- python3 scripts/time_ops.py --configs C5,C5b32,C5x8b32,C5vb32 --iters 20 --tag wide$v > $OUT/time_$v.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/time_$v.txt; exit $rc; }
  grep '{' $OUT/time_$v.txt
done
for v in 1 0; do echo "== $v"; cut -d, -f1-4 $OUT/trace_$v/run_kernel_stats.csv | grep -v distribution | head -6; done
