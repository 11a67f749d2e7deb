#!/bin/bash
# Round 4, GPU call O: the merged box pass (option box_merge: both leaf slots' box tests dealt
# out over the wave's lanes) -- parity (scenes and the adversarial box cases with it on), then an
# interleaved A/B against the default on scene 8 at 1080p and the stats twin with it on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "gpurun_out/$name.log" | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
step pytest_bm 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -k "box_merge or adversarial_case" -rf
step ab_bm 300 python -u tools/option_ab.py --specs default,box_merge=1 --scene 8 --rounds 7
step kstats_bm 200 python tools/kernel_stats.py --scene 8 --frames 64 --options '{"box_merge": 1}'
exit 0
