#!/bin/bash
# Round 3, GPU call B: the gallery seed spread through the reference's PNG pipeline, and the
# region timers of the stats build (A/B library) on scenes 8, 0, 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step seed_probe_png 400 python -u tools/gallery_seed_probe.py
step kstats_s8 200 python -u tools/kernel_stats.py --scene 8 --frames 64
step kstats_s0 200 python -u tools/kernel_stats.py --scene 0 --frames 64
step kstats_s6 200 python -u tools/kernel_stats.py --scene 6 --frames 64
exit 0
