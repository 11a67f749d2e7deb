#!/bin/bash
# Round 3, GPU call F: the two-level walk with its leaf records in LDS -- the GPU suite's
# adversarial tests, then the BVH scaling probe (leaf records in LDS vs global).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_adv 400 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -rf
step bvh_scaling 500 python -u tools/bvh_scaling.py
exit 0
