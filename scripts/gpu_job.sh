#!/bin/bash
# One parameterised GPU job runner (replaces the per-call scripts of rounds
# 1-5, listed with what each produced in scripts/README.md).
#
#   bash scripts/gpu_job.sh TAG STEP [STEP ...]
#
# Every step runs under its own time limit and writes under gpurun_out/TAG/;
# the first failing step ends the job (no GPU work after a fault, an abort or
# a time-limit kill).  Steps:
#   tests[=PATTERN]      python -m pytest tests -m gpu (-k PATTERN)
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         python bench.py ARGS (comma-separated args: bench=--stripes,128)
#   trace[=ARGS]         rocprofv3 --kernel-trace --stats of bench.py --no-cpu --no-single
#                        --no-unpadded --no-other --no-host ARGS
#   ops=CFG              rocprofv3 kernel trace of scripts/time_ops.py --configs CFG
#   pmc=COUNTERS[@ARGS]  one rocprofv3 --pmc pass (COUNTERS comma-separated) over bench.py
#                        --no-cpu --no-single --no-unpadded --no-other --no-host ARGS
#   sweep=ARGS           python scripts/c3_tpw_sweep.py ARGS (comma-less args split on ':')
#   probe                scripts/micro/launch_probe (C driver: host vs GPU time per call)
#   py=SCRIPT[@ARGS]     python SCRIPT ARGS (ARGS split on ':')
#   pmcpy=COUNTERS@SCRIPT[@ARGS]  one rocprofv3 --pmc pass over python3 SCRIPT ARGS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
QUIET="--no-cpu --no-single --no-unpadded --no-other --no-host"
n=0
run() {  # run LIMIT NAME CMD...: one step, its own time limit and log
  local lim=$1 name=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "step $name rc=$rc"
  tail -3 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
for step in "$@"; do
  n=$((n + 1))
  key=${step%%=*}
  val=""
  [ "$step" != "$key" ] && val=${step#*=}
  case $key in
    tests)
      if [ -n "$val" ]; then run 900 "$n-tests" python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$val"
      else run 900 "$n-tests" python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread; fi ;;
    smoke) run 300 "$n-smoke" python -c 'import __graft_entry__ as g; g.smoke()' ;;
    bench) run 600 "$n-bench" python bench.py ${val//,/ } ;;
    trace) run 300 "$n-trace" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace$n" -o run -- python3 bench.py $QUIET ${val//,/ } ;;
    ops) run 300 "$n-ops" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ops$n" -o run -- python3 scripts/time_ops.py --configs "$val" --iters 20 ;;
    pmc)
      ctr=${val%%@*}
      args=""
      [ "$val" != "$ctr" ] && args=${val#*@}
      run 300 "$n-pmc" rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$OUT/pmc$n" -o run -- python3 bench.py $QUIET --steps 50 --warmup 5 ${args//,/ } ;;
    sweep) run 600 "$n-sweep" python3 scripts/c3_tpw_sweep.py ${val//:/ } ;;
    probe) run 120 "$n-probe" scripts/micro/launch_probe ;;
    pmcpy)
      ctr=${val%%@*}
      rest=${val#*@}
      scr=${rest%%@*}
      args=""
      [ "$rest" != "$scr" ] && args=${rest#*@}
      run 300 "$n-pmcpy" rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$OUT/pmc$n" -o run -- python3 "$scr" ${args//:/ } ;;
    py)
      scr=${val%%@*}
      args=""
      [ "$val" != "$scr" ] && args=${val#*@}
      run 600 "$n-py" python3 "$scr" ${args//:/ } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
