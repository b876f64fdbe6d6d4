#!/bin/bash
# Round 5, call g: C3 tiles-per-workgroup sweep (strided tpwN: tile b + i*grid;
# contiguous cpwN: tiles b*N .. b*N+N-1), 256 and 16 stripes per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5g; mkdir -p $OUT; : > $OUT/ab.log
L=$PWD/labbuild
for pass in 1 2; do
  for v in prod:$PWD/reedsolomon16_amd/librs_mi355x.so tpw3:$L/tpw3/librs_mi355x.so tpw4:$L/tpw4/librs_mi355x.so tpw6:$L/tpw6/librs_mi355x.so tpw8:$L/tpw8/librs_mi355x.so tpw16:$L/tpw16/librs_mi355x.so cpw4:$L/cpw4/librs_mi355x.so cpw8:$L/cpw8/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    for st in 256 16; do
      echo -n "$n $st " >> $OUT/ab.log
      RS_MI355X_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-other --no-host --no-single --steps 30 --warmup 5 --stripes $st >> $OUT/ab.log 2> $OUT/ab_$n.err || { tail -3 $OUT/ab_$n.err; exit 1; }
    done
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r5g/ab.log"):
    tag, st, js = line.split(" ", 2)
    d = json.loads(js)
    print(tag, st, d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["unpadded_rows"]["frac"])
PY
