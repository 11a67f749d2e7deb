#!/bin/bash
# Round 4, GPU call AI: the leaf tests at wave priority 2 inside the rounds (walk 1, shading 0)
# (lib/alt) against the shipped form (lib/librtamd.so); scenes 8 / 0 / 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step prio_leaf2 500 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/alt/librtamd.so,raytracing-book_amd/lib/librtamd.so --scenes 8,0,6 --rounds 7
exit 0
