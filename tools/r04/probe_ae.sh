#!/bin/bash
# Round 4, GPU call AE: wave priority placements against the previous library (lib/prev, no
# s_setprio): the walk at 1 (v_w1), the walk at 3 (v_w3), the leaf tests at 1 (v_leaf); scenes 8 / 0 / 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
L=raytracing-book_amd/lib
step prio_ab2 700 python -u tools/lib_ab.py --libs $L/prev/librtamd.so,$L/v_w1/librtamd.so,$L/v_w3/librtamd.so,$L/v_leaf/librtamd.so --scenes 8,0,6 --rounds 7
exit 0
