#!/bin/bash
# Round 5, call o: bit-plane XORs as compiler builtins instead of inline asm
# (the asm boundaries cost hazard s_nops and blocked folding: C4 decoder
# 12444 -> 11926 instructions, C3 17790 -> 16221): parity, then C3 / C4
# timing against the asm build (labbuild/base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5o; mkdir -p $OUT; : > $OUT/time.log; : > $OUT/c3.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bsdec.py tests/test_gpu_bitslice.py tests/test_gpu_golden.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in asm:$PWD/labbuild/base/librs_mi355x.so bi:$PWD/reedsolomon16_amd/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 scripts/time_ops.py --configs C4x16,C4,C4e1 --iters 20 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
    RS_MI355X_LIB=$lib timeout -k 10 200 python3 scripts/c3_tpw_sweep.py --stripes 256 --slices 1,8 --tiles 0 --steps 0 --iters 20 | sed "s/^{/{\"tag\": \"$n\", /" >> $OUT/c3.log 2> $OUT/$n.c3err || { tail -3 $OUT/$n.c3err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/time.log'):
    d=json.loads(l); print(d['tag'], d['config'], d['us'])
for l in open('$OUT/c3.log'):
    d=json.loads(l); print(d['tag'], 'C3', d['stripes'], d['ranks'], d['ms'], d['frac'])"
