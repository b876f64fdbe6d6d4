#!/bin/bash
# GPU suite, then C5 encode with the final FFT in subfield coordinates vs full field (RS_NO_SUB=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c5sub; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for v in sub full; do
  if [ $v = full ]; then export RS_NO_SUB=1; else unset RS_NO_SUB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$v -o run -- python3 scripts/time_ops.py --configs C5,C5x8,C4x16 --iters 20 --tag $v > $OUT/time_$v.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/time_$v.txt; exit $rc; }
  grep '{' $OUT/time_$v.txt
done
for v in sub full; do echo "== $v"; cut -d, -f1-4 $OUT/trace_$v/run_kernel_stats.csv | head -5; done
