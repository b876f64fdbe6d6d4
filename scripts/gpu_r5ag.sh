#!/bin/bash
# Round 5, call ag: packed units in the encoder's 128-byte LDS tiles (LTile PK
# for W = 4: low 16 | high 16 bytes, rows still padded by 16): parity, then
# C5 encode / verify timing against the split layout (labbuild/base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5ag; mkdir -p $OUT; : > $OUT/time.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_stream.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for v in base:$PWD/labbuild/base/librs_mi355x.so pack:$PWD/reedsolomon16_amd/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    RS_MI355X_LIB=$lib timeout -k 10 200 python3 scripts/time_ops.py --configs C5b32,C5vb32,C5 --iters 10 --tag $n >> $OUT/time.log 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/time.log'):
    d=json.loads(l); print(d['tag'], d['config'], d['us'])"
