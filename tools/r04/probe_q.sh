#!/bin/bash
# Round 4, GPU call Q: the quad and light tables in LDS (part of option shade_lds) -- the parity
# tests that cover the shading tables, then the new library against the previous one (lib/prev:
# the sphere / box / texture tables only) on scenes 6 / 7 / 8 / 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -9 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_ql 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -rf -k "shading_tables or kernel_matches"
step lib_ab_ql 500 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/prev/librtamd.so --scenes 6,7 --rounds 9
exit 0
