#!/bin/bash
# Round 6, call d: row stagger (bytes between rows beyond the row) for the
# per-rank slices of a byte-range split: the stagger is the rank's own
# allocation choice, tuned in round 4 for full 1 MiB rows only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6d
mkdir -p $OUT
PADS=0,512,1024,1536,2048,2560,3072,3584,4096,4608,5632,6656,7680,9728,11776
for sl in 8 4 2 1; do
  timeout -k 10 300 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices $sl --tiles 0,1 --pad $PADS --iters 20 > $OUT/pad_s$sl.jsonl 2> $OUT/pad_s$sl.err
  rc=$?; echo "slice $sl rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r6d/pad_s*.jsonl")):
    for l in open(f):
        d=json.loads(l); print(d["ranks"], d["tiles"], d["pad"], d["frac"])
PY
