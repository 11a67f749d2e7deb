#!/bin/bash
# Round 4, GPU call I: the two-level walk with gathered global steps (option tl_gather) and the
# best-first node order (option tl_order) --
# the forced-split parity test (every cap x gather form, bit for bit against the oracle), then
# the 4000-sphere cloud at the forced caps and the 9000-sphere cloud for gather 0 / 8 / 32 and the
# breadth-first / best-first node order (option tl_order).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_tl 400 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -k two_level -rf
step bvh_gather 700 python -u tools/bvh_scaling.py --gather 0,8,32 --orders 0,1 --no-tll0 --sizes 4000,9000
exit 0
