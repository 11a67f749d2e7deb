#!/bin/bash
# Round 4, GPU call Y: the partial walk's stop check every 3rd node step (default) against every
# 2nd (lib/alt2) and every 4th (lib/alt4), under the per-BVH walk thresholds, scenes 6 / 7 / 0 / 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step unroll_ab 600 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/alt2/librtamd.so,raytracing-book_amd/lib/alt4/librtamd.so --scenes 6,7,0,8 --rounds 5
exit 0
