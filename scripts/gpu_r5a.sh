#!/bin/bash
# Round 5, call a: GPU suite (stream mirrors first), C3 A/B of the idle
# last-chunk prefetch (labbuild/old = round-4 kernel), then the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py > $OUT/pytest_stream.log 2>&1
rc=$?; echo "stream pytest rc=$rc"; tail -3 $OUT/pytest_stream.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/ab.log
for pass in 1 2; do
  for v in old:$PWD/labbuild/old/librs_mi355x.so new:$PWD/reedsolomon16_amd/librs_mi355x.so xcd:$PWD/labbuild/xcd/librs_mi355x.so stripe:$PWD/labbuild/stripe/librs_mi355x.so xcd2:$PWD/labbuild/xcd2/librs_mi355x.so; do
    n=${v%%:*}; lib=${v#*:}
    echo -n "$n " >> $OUT/ab.log
    RS_MI355X_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu --no-other --no-host --no-single --no-unpadded --steps 30 --warmup 5 >> $OUT/ab.log 2> $OUT/ab_$n.err || { tail -3 $OUT/ab_$n.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/r5a/ab.log"):
    tag, js = line.split(" ", 1)
    d = json.loads(js)
    print(tag, d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; tail -c 3000 $OUT/bench.json; exit $rc
