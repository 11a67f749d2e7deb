#!/bin/bash
# Round 4, GPU call Z: the walk round threshold on the big clouds (4000 spheres all in LDS and at the
# 32 KB cap; the 9000-sphere cloud, two-level by itself): walk_frac 32 / 48 (default) / 64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "cost_vs\|9000" "gpurun_out/$name.log" | cut -c1-220; [ $rc -eq 0 ] || exit $rc; }
step bvh_wf32 300 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 32768 --extra '{"walk_frac": 32}'
step bvh_wf48 300 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 32768 --extra '{"walk_frac": 48}'
step bvh_wf64 300 python -u tools/bvh_scaling.py --sizes 4000,9000 --no-tll0 --caps 32768 --extra '{"walk_frac": 64}'
exit 0
