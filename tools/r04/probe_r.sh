#!/bin/bash
# Round 4, GPU call R: min / max through the compiler builtins instead of inline asm (no hazard
# s_nops in the node step; ray_t canonicalized once per walk) -- the GPU suite, then the new
# library against the previous one (lib/prev, inline asm) on scenes 8 / 0 / 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -9 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf
step lib_ab_mm 500 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/prev/librtamd.so --scenes 8,0,6 --rounds 7
exit 0
