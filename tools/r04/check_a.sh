#!/bin/bash
# Round 4, GPU call A: HEAD check after the boundary fixes -- the GPU suite (with the new
# full-size walk/schedule option tests and the sm_frac test), the default bench line
# (CPU baseline on the quota's threads, native gather path) and rocprof of the C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf
step bench 400 python -u bench.py
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
exit 0
