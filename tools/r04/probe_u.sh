#!/bin/bash
# Round 4, GPU call U: walk_frac for the non-compact-box kernels (scenes 0 and 6; call T: 40 beat the
# default 48 on both) at 32 / 36 / 40 / 44, and scene 8's (compact-box kernel) at 44 / 52.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step knobs3_s0 400 python -u tools/option_ab.py --specs "default,walk_frac=32,walk_frac=36,walk_frac=40,walk_frac=44" --scene 0 --rounds 7
step knobs3_s6 400 python -u tools/option_ab.py --specs "default,walk_frac=32,walk_frac=36,walk_frac=40,walk_frac=44" --scene 6 --rounds 7
step knobs3_s8 400 python -u tools/option_ab.py --specs "default,walk_frac=44,walk_frac=52" --scene 8 --rounds 7
exit 0
