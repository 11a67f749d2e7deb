#!/bin/bash
# Round 4, GPU call AF: wave priority, walk and leaf tests above shading: both at 1 (v_both), walk 2 /
# leaf 1 (v_w2l1), against the walk alone at 1 (v_w1) and no s_setprio (lib/prev); scenes 8 / 0 / 6 / 7.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
L=raytracing-book_amd/lib
step prio_ab3 800 python -u tools/lib_ab.py --libs $L/prev/librtamd.so,$L/v_w1/librtamd.so,$L/v_both/librtamd.so,$L/v_w2l1/librtamd.so --scenes 8,0,6,7 --rounds 7
exit 0
