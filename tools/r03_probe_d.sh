#!/bin/bash
# Round 3, GPU call D: the GPU suite, then scene 8 / 0 timings of the default path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf --durations=10
step ab_s8 200 python -u tools/option_ab.py --specs default,spine=0 --scene 8
step ab_s6 200 python -u tools/option_ab.py --specs default,compact_boxes=0 --scene 6
exit 0
