#!/bin/bash
# Round 4, GPU call AG: the walk + leaf rounds at wave priority 1 as one region (the shipped form)
# -- the GPU suite, then against no s_setprio (lib/prev) and the two-site form of call AF
# (lib/v_both_prev) on scenes 8 / 0 / 6 / 7.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER\|passed" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
L=raytracing-book_amd/lib
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step prio_ab4 800 python -u tools/lib_ab.py --libs $L/librtamd.so,$L/prev/librtamd.so,$L/v_both_prev/librtamd.so --scenes 8,0,6,7 --rounds 7
exit 0
