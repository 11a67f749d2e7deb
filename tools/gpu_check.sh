#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a step that faults/aborts/times out
# (exit status other than 0 or 1) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"tests smoke bench prof"}
run() {   # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail=25 -rf --durations=20 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    ab)    run ab 600 python tools/ab_variants.py ${AB_ARGS:-} ;;
    stats) run kstats 300 python tools/kernel_stats.py ${STATS_ARGS:-} ;;
    list)  run pmc_list 120 rocprofv3 -L ;;
    pmc)   run pmc 900 python tools/pmc_profile.py ${PMC_ARGS:-} ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:-} ;;
  esac
done
exit 0
