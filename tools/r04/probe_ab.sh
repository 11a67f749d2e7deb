#!/bin/bash
# Round 4, GPU call AB: every exact layout / shortcut option of the release library turned off in
# turn on scenes 8 and 6, against the default, after the round's changes (does each default still pay?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step offs_s8 500 python -u tools/option_ab.py --specs "default,box_pretest=0,fastdiv=0,spine=0,perlin_packed=0,sparse_stage=0,leaf_prefetch=0,shade_lds=0,compact_boxes=0" --scene 8 --rounds 3
step offs_s6 500 python -u tools/option_ab.py --specs "default,box_pretest=0,fastdiv=0,sparse_stage=0,shade_lds=0,sphere_pairs=0" --scene 6 --rounds 3
exit 0
