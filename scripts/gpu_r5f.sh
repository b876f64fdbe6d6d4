#!/bin/bash
# Round 5, call f: C3 tiles per workgroup -- one (product) against 2, 4 and a
# persistent 512-workgroup grid (the kernel's next-tile prefetch is live then).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5f; mkdir -p $OUT; : > $OUT/ab.log
for pass in 1 2; do
  for v in prod:$PWD/reedsolomon16_amd/librs_mi355x.so tpw2:$PWD/labbuild/tpw2/librs_mi355x.so tpw4:$PWD/labbuild/tpw4/librs_mi355x.so pers:$PWD/labbuild/pers/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    echo -n "$n " >> $OUT/ab.log
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-other --no-host --no-single --steps 30 --warmup 5 >> $OUT/ab.log 2> $OUT/ab_$n.err || { tail -3 $OUT/ab_$n.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r5f/ab.log"):
    tag, js = line.split(" ", 1)
    d = json.loads(js)
    print(tag, d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["unpadded_rows"]["frac"])
PY
