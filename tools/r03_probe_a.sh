#!/bin/bash
# Round 3, GPU call A: the gallery seed spread, the BVH scaling of the
# two-level walk (item 4), the rocprof kernel stats of the C3 bench and its PMC passes.
# Every step has its own time limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step seed_probe 400 python -u tools/gallery_seed_probe.py
step bvh_scaling 300 python -u tools/bvh_scaling.py
step rocprof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_c3 -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline
step pmc_c3 400 python tools/pmc_profile.py --groups 0,2,3,4,15 --target "--scene 8 --frames 64" --valu-key scene8_1920x1080_f64_d5 --traffic-key scene8_1920x1080_f64_d5 --out gpurun_out/pmc_c3.json
exit 0
