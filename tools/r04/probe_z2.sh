#!/bin/bash
# Round 4, GPU call Z2: the walk round threshold on the big clouds (4000 spheres all in LDS and at the
# 32 KB cap; the 9000-sphere cloud, two-level by itself): walk_frac 16 / 24 (call Z: 32 beat 48 on the two-level walks, 48 beat 32 all in LDS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "cost_vs\|9000" "gpurun_out/$name.log" | cut -c1-220; [ $rc -eq 0 ] || exit $rc; }
step bvh_wf16 300 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 32768 --extra '{"walk_frac": 16}'
step bvh_wf24 300 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 32768 --extra '{"walk_frac": 24}'
exit 0
