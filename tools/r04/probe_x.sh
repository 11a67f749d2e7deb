#!/bin/bash
# Round 4, GPU call X: the shading threshold (sm_frac; by kernel: 50 compact-box, 56 else) and
# batch (sm_batch, 64) re-swept under the per-BVH walk thresholds, on scenes 6 / 7 / 0 / 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step sm_s6 300 python -u tools/option_ab.py --specs "default,sm_frac=48,sm_frac=60,sm_frac=64,sm_batch=48" --scene 6 --rounds 5
step sm_s7 300 python -u tools/option_ab.py --specs "default,sm_frac=48,sm_frac=60,sm_frac=64,sm_batch=48" --scene 7 --rounds 5
step sm_s0 300 python -u tools/option_ab.py --specs "default,sm_frac=52,sm_frac=60,sm_batch=48" --scene 0 --rounds 5
step sm_s8 300 python -u tools/option_ab.py --specs "default,sm_frac=46,sm_frac=54,sm_batch=48" --scene 8 --rounds 5
exit 0
