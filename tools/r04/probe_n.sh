#!/bin/bash
# Round 4, GPU call N: the phased two-level walk (option tl_gather = G: LDS steps for the lanes in
# the LDS prefix with no per-step source test, then a global phase as soon as G lanes wait at a
# global node) for G = 1, 4 against the per-step test (0), and the mixed step (option tl_mixed: an LDS
# step, then a wave-uniform global step) -- parity, then the cloud caps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep cost_vs "gpurun_out/$name.log" | cut -c1-200; tail -2 "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step pytest_tl 400 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -k two_level -rf
step bvh_phase 600 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --gather 0,1,4 --caps 130048,98304,32768,8192
step bvh_mixed 400 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 130048,98304,32768,8192 --extra '{"tl_mixed": 1}'
exit 0
