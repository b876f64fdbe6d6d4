#!/bin/bash
# Stripes per launch at full rows and at the 2- and 8-rank byte-range slices
# (one GPU, --slice-of), 3.5 KiB row stagger: does a larger batch shrink the
# slices' fill/drain share?  Output: gpurun_out/r4t/batch.jsonl
set -o pipefail
mkdir -p gpurun_out/r4t
out=gpurun_out/r4t/batch.jsonl
: > $out
for sl in 0 2 8; do
  for B in 128 256 512; do
    if [ $sl = 0 ] && [ $B = 512 ]; then continue; fi
    timeout -k 10 240 python bench.py --steps 100 --warmup 10 --stripes $B --slice-of $sl --no-cpu --no-single --no-unpadded --no-other > gpurun_out/r4t/one.json || { echo "bench sl=$sl B=$B failed rc=$?"; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/r4t/one.json').read().strip().splitlines()[-1])
print(json.dumps({'slice_of':$sl,'stripes':$B,'kernel_ms':d['roofline']['kernel_ms'],'frac':d['roofline']['frac'],'value':d['value']}))" >> $out
    tail -1 $out
  done
done
