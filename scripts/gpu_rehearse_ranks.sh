#!/bin/bash
# N-rank bench rehearsal on a one-GPU box: the same rank code as the driver's
# N-GPU run (torch.distributed.run launch, per-rank byte ranges, max-over-ranks
# timing, rank-0 JSON line), with a gloo process group and every rank on GPU 0
# (bench.py --backend gloo).  The rates are meaningless (the ranks share one
# GPU); the point is that every layout runs to its JSON line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rehearse
rm -rf $OUT; mkdir -p $OUT
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --backend gloo --stripes 16 --steps 10 --warmup 2 --no-host --no-cpu > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?; echo "$n rc=$rc"; tail -c 700 $OUT/$n.json; echo; [ $rc -eq 0 ] || { tail -20 $OUT/$n.err; exit $rc; }
}
run g2_bytes_weak --gpus 2 && run g4_bytes_weak --gpus 4 && run g2_bytes --gpus 2 --split bytes && \
run g2_stripes --gpus 2 --split stripes && run g2_c5 --gpus 2 --workload C5
