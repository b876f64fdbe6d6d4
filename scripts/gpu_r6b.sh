#!/bin/bash
# Round 6, call b: L2 <-> fabric counters of the C3 encode for the tile maps
# (one tile per workgroup vs four a grid apart), full rows and the 8-rank
# slice, to find what the distant tiles change.
# Each pass is its own rocprofv3 run (<= 4 TCC counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6b
mkdir -p $OUT
P1="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
P2="TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum"
P3="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum"
for cfg in "full1 256 1 1" "full4 256 1 4" "sl8t1 256 8 1" "sl8t4 256 8 4" "sl8big 2048 8 4"; do
  set -- $cfg
  name=$1; B=$2; SL=$3; T=$4
  timeout -k 10 120 python3 scripts/c3_tpw_sweep.py --stripes $B --slices $SL --tiles $T --iters 20 > $OUT/time_$name.json 2> $OUT/time_$name.err
  rc=$?; echo "time $name rc=$rc $(cat $OUT/time_$name.json)"; [ $rc -eq 0 ] || exit $rc
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_${name}_$i -o run -- python3 scripts/c3_tpw_sweep.py --stripes $B --slices $SL --tiles $T --iters 5 > /dev/null 2> $OUT/pmc_${name}_$i.err
    rc=$?; echo "pmc $name $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/pmc_summary.py $OUT k_encode_hp > $OUT/summary.txt; cat $OUT/summary.txt
