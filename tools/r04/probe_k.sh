#!/bin/bash
# Round 4, GPU call K: the two-level node read without the register hazard (rt_kernel.hip
# load_node: a wave-uniform test for the plain LDS step, global and LDS reads into registers of
# their own otherwise) -- forced-split parity, then the 4000-sphere cloud at caps from 31 global
# nodes to 256 LDS nodes and the 9000-sphere cloud.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -12 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_tl 400 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -k two_level -rf
step bvh_caps 500 python -u tools/bvh_scaling.py --sizes 4000,9000 --caps 130048,98304,65536,32768,8192
exit 0
