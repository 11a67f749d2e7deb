#!/bin/bash
# Round 4, GPU call T: the non-compact-box kernels' shading threshold (sm_frac, default 56) and walk
# threshold (walk_frac, default 48) around the scene 6 optimum of call S, on scenes 6 and 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step knobs2_s6 400 python -u tools/option_ab.py --specs "default,sm_frac=60,sm_frac=64,sm_frac=60;walk_frac=40,walk_frac=40" --scene 6 --rounds 7
step knobs2_s0 400 python -u tools/option_ab.py --specs "default,sm_frac=60,sm_frac=64,sm_frac=60;walk_frac=40,walk_frac=40" --scene 0 --rounds 7
exit 0
