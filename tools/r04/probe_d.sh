#!/bin/bash
# Round 4, GPU call D: leaf record prefetch (option leaf_prefetch) -- parity, A/B on scene 8 at
# 1080p and 4K (and scene 0 / 6, which do not take it: must be unchanged).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_pf 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 120 --timeout-method thread -rf -k "prefetch"
step pf_s8 300 python -u tools/option_ab.py --scene 8 --rounds 9 --specs default,leaf_prefetch=0
step pf_s8_4k 300 python -u tools/option_ab.py --scene 8 --rounds 5 --width 3840 --height 2160 --specs default,leaf_prefetch=0
step pf_s8_b 300 python -u tools/option_ab.py --scene 8 --rounds 9 --specs leaf_prefetch=0,default
exit 0
