#!/bin/bash
# Round 4, GPU call F: the two-level walk's subtree-ordered global nodes (option tl_dfs) --
# parity (forced splits vs the oracle, and the 9000-sphere cloud's own two-level launch through the
# adversarial suite) and tools/bvh_scaling.py with the layout on and off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_tl 300 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -q -x --timeout 200 --timeout-method thread -rf
step bvh_scaling 600 python -u tools/bvh_scaling.py
exit 0
