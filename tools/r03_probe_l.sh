#!/bin/bash
# Round 3, GPU call L: sparse vs dense staging inside the same library (scenes 6 / 8 / 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step ab_sp_s6 300 python -u tools/option_ab.py --specs default,sparse_stage=0 --scene 6 --rounds 7
step ab_sp_s8 300 python -u tools/option_ab.py --specs default,sparse_stage=0 --scene 8 --rounds 7
step ab_sp_s0 300 python -u tools/option_ab.py --specs default,sparse_stage=0 --scene 0 --rounds 7
exit 0
