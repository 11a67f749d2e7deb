#!/bin/bash
# Round 4, GPU call J: the two-level walk's fixed cost -- the 4000-sphere cloud with all but a few
# dozen nodes (cap 130048 B: 31 nodes global, the last of the deepest level), all but 1/16, and
# the usual caps, against all in LDS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -8 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step bvh_caps 400 python -u tools/bvh_scaling.py --sizes 4000 --no-tll0 --caps 130048,122880,98304,32768
exit 0
