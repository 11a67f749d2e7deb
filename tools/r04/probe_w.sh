#!/bin/bash
# Round 4, GPU call W: walk_frac on the small-BVH scenes (6 and 7: 7 nodes; 9: 3 nodes) down to 4,
# where call V found scene 6 still improving at 16 (-6%).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step knobs5_s6 400 python -u tools/option_ab.py --specs "default,walk_frac=4,walk_frac=8,walk_frac=12,walk_frac=16" --scene 6 --rounds 7
step knobs5_s7 400 python -u tools/option_ab.py --specs "default,walk_frac=8,walk_frac=16,walk_frac=32" --scene 7 --rounds 7
step knobs5_s9 400 python -u tools/option_ab.py --specs "default,walk_frac=8,walk_frac=16,walk_frac=32" --scene 9 --rounds 7
exit 0
