#!/bin/bash
# Round 3, GPU call J: 5 waves per SIMD (640-thread workgroups, 96 VGPRs) against the default
# shape on scenes 8 / 0 / 6; the Perlin corner weights simplified (working tree vs HEAD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf
step ab_w5_s8 300 python -u tools/option_ab.py --specs default,waves5=1 --scene 8 --rounds 5
step ab_w5_s0 300 python -u tools/option_ab.py --specs default,waves5=1 --scene 0 --rounds 5
step ab_w5_s6 300 python -u tools/option_ab.py --specs default,waves5=1 --scene 6 --rounds 5
step lib_ab 400 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/librtamd_head.so --scenes 8,3 --rounds 7
exit 0
