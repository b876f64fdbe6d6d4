#!/bin/bash
# 8-rank byte-range slice (128 KiB of every row) and full rows: batch size and row stagger.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/slice
for st in 64 128 256; do
  timeout -k 10 200 python scripts/time_pad.py --S 131072 --stripes $st --pads 0,3072,1024,0,3072 --iters 40 > gpurun_out/slice/s128k_$st.log 2>&1
  rc=$?; echo "slice stripes=$st rc=$rc"; grep row_pad gpurun_out/slice/s128k_$st.log; [ $rc -eq 0 ] || exit $rc
done
for st in 32 128 256; do
  timeout -k 10 300 python scripts/time_pad.py --stripes $st --pads 3072,0,3072 --iters 20 > gpurun_out/slice/s1m_$st.log 2>&1
  rc=$?; echo "full stripes=$st rc=$rc"; grep row_pad gpurun_out/slice/s1m_$st.log; [ $rc -eq 0 ] || exit $rc
done
