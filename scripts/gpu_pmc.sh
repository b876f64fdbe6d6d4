#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) on the profiling driver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_OUT:-pmc}
mkdir -p $OUT
ARGS="${PROF_ARGS:---iters 10}"
i=0
IFS='|'
for pmc in $PMC_SETS; do
  i=$((i+1))
  IFS=' '
  timeout -k 10 180 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o run -- python3 scripts/prof_encode.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc$i ($pmc) rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  IFS='|'
done
exit 0
