#!/bin/bash
# Radix-16 LDS kernels: their parity tests, the GPU suite, then C4 / C5 kernel
# times under rocprofv3 with the radix-16 kernels on (default) and off (RS_R16=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r16
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k radix16 -x -v --timeout 120 --timeout-method thread > gpurun_out/r16/pytest_r16.log 2>&1
rc=$?; tail -4 gpurun_out/r16/pytest_r16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r16/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r16/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r16/times.log
for mode in on off; do
  if [ $mode = off ]; then export RS_R16=0; else unset RS_R16; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r16/$mode -o run -- python3 scripts/time_ops.py --configs C4,C4e1,C5,C5x8 --iters 30 --tag $mode > gpurun_out/r16/$mode.out 2> gpurun_out/r16/$mode.err
  rc=$?; [ $rc -eq 0 ] || { echo "fail $mode rc=$rc"; tail -5 gpurun_out/r16/$mode.err; exit $rc; }
  python3 - "$mode" >> gpurun_out/r16/times.log <<'PY'
import csv, glob, sys
m = sys.argv[1]
f = glob.glob(f"gpurun_out/r16/{m}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "_lds" in r["Name"] or "_r16" in r["Name"]:
        print(m, r["Name"][:60], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
  cat gpurun_out/r16/$mode.out >> gpurun_out/r16/times.log
done
cat gpurun_out/r16/times.log
