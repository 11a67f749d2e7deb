#!/bin/bash
# Round 3, GPU call G: the packed Perlin table -- GPU suite, the working tree's library against
# HEAD's (tools/build_rev.sh HEAD head), and the shading ablations (A/B build: d1 Perlin
# constant, d2 image texture constant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf
step lib_ab 400 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/librtamd_head.so --scenes 8,0,6 --rounds 7
step ablate 300 python -u tools/ab_variants.py --variants 0,0d1,0d2 --scene 8 --rounds 5
exit 0
