#!/bin/bash
# Round 4, GPU call S: the scheduling thresholds re-swept on the current kernel (walk_frac: a walk
# round stops when this many 64ths of its lanes hold a leaf; sm_frac: shading once this many 64ths
# of the walking lanes are done) on scenes 8 and 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step knobs_s8 400 python -u tools/option_ab.py --specs default,walk_frac=40,walk_frac=56,sm_frac=44,sm_frac=56 --scene 8 --rounds 5
step knobs_s6 400 python -u tools/option_ab.py --specs default,walk_frac=40,walk_frac=56,sm_frac=50,sm_frac=60 --scene 6 --rounds 5
exit 0
