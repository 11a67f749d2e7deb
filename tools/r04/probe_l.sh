#!/bin/bash
# Round 4, GPU call L: the two-level walk with the small sphere / box tables staged beside the
# top levels (option tl_small_lds, default 1) against without (0) -- forced-split parity, then
# the 4000-sphere cloud at caps from 31 global nodes to 256 LDS nodes and the 9000-sphere cloud.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -7 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_tl 400 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -k two_level -rf
step bvh_small1 500 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 130048,98304,65536,32768,8192
step bvh_small0 500 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 130048,98304,65536,32768,8192 --extra '{"tl_small_lds": 0}'
exit 0
