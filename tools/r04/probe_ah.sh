#!/bin/bash
# Round 4, GPU call AH: the path starts (sample claims, camera rays) at wave priority 1 too, so only
# shading runs at 0, against the shipped form (lib/prev); scenes 8 / 0 / 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step prio_start 500 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/prev/librtamd.so --scenes 8,0,6 --rounds 7
exit 0
