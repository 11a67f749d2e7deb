#!/bin/bash
# Round 3, GPU call C: the spine entry (adversarial parity + A/B timing on scenes 8, 0, 6),
# the gallery's sample count from its pixel noise, and the region timers with the entry on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step adversarial 400 python -u -m pytest tests/test_gpu_adversarial.py -x -q --timeout 300 --timeout-method thread
step spine_ab_s8 200 python -u tools/option_ab.py --specs default,spine=0 --scene 8
step spine_ab_s0 200 python -u tools/option_ab.py --specs default,spine=0 --scene 0
step gallery_spp 300 python -u tools/gallery_spp_probe.py 6 1
step kstats_s8 200 python -u tools/kernel_stats.py --scene 8 --frames 64
exit 0
