#!/bin/bash
# Round 4, GPU call AC: a separate walk threshold for rounds whose walking lanes are mostly camera
# rays (option walk_frac_cam) on scenes 8 / 0 / 6: 24 / 40 / 56 / 64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step wfc_s8 300 python -u tools/option_ab.py --specs "default,walk_frac_cam=24,walk_frac_cam=40,walk_frac_cam=56,walk_frac_cam=64" --scene 8 --rounds 5
step wfc_s0 300 python -u tools/option_ab.py --specs "default,walk_frac_cam=16,walk_frac_cam=48,walk_frac_cam=64" --scene 0 --rounds 5
step wfc_s6 300 python -u tools/option_ab.py --specs "default,walk_frac_cam=24,walk_frac_cam=48" --scene 6 --rounds 5
exit 0
