#!/bin/bash
# Round 4, GPU call AA: the staged launch's unit split (staged_chunk_target: chunks per resident
# wave, default 48) on scenes 8 / 6 / 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep median "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step sct_s8 300 python -u tools/option_ab.py --specs "default,staged_chunk_target=24,staged_chunk_target=96" --scene 8 --rounds 5
step sct_s6 300 python -u tools/option_ab.py --specs "default,staged_chunk_target=24,staged_chunk_target=96" --scene 6 --rounds 5
step sct_s0 300 python -u tools/option_ab.py --specs "default,staged_chunk_target=24,staged_chunk_target=96" --scene 0 --rounds 5
exit 0
