#!/bin/bash
# Round 4, GPU call E: both leaf slots' records prefetched at once (working tree) against one
# slot at a time (HEAD, lib/prev) -- scenes 8 (takes it) and 0 / 6 (do not: equal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step lib_ab 400 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/prev/librtamd.so --scenes 8,0 --rounds 9
exit 0
