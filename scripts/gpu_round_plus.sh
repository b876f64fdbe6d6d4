#!/bin/bash
# Round evidence (scripts/gpu_round.sh), then C4/C5 kernel times at both LDS tile widths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_round.sh || exit $?
for w in wide narrow; do
  RS_UNIT_WIDTH=$w timeout -k 10 200 python scripts/time_ops.py --configs C4,C5,C5x8 --iters 40 --tag $w > gpurun_out/round/width_$w.log 2>&1
  rc=$?; echo "width $w rc=$rc"; grep '{' gpurun_out/round/width_$w.log; [ $rc -eq 0 ] || exit $rc
done
