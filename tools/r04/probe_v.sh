#!/bin/bash
# Round 4, GPU call V: walk_frac for the non-compact-box kernels (scenes 0 and 6) below 32, where call U
# still improved scene 6: 16 / 20 / 24 / 28 / 32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step knobs4_s6 400 python -u tools/option_ab.py --specs "default,walk_frac=16,walk_frac=20,walk_frac=24,walk_frac=28,walk_frac=32" --scene 6 --rounds 7
step knobs4_s0 400 python -u tools/option_ab.py --specs "default,walk_frac=20,walk_frac=24,walk_frac=28,walk_frac=32" --scene 0 --rounds 7
exit 0
