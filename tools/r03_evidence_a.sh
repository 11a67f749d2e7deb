#!/bin/bash
# Round-3 final evidence, part A: GPU tests, then the PMC passes per config (VALU count,
# lane utilisation, DRAM bytes) whose profiles/valu.json the bench lines of part B read.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step pmc_c3 300 python tools/pmc_profile.py --groups 0,2,3,4,5,15 --target "--scene 8 --frames 64" --valu-key scene8_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c3.json
step pmc_c2 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 0 --frames 64 --spp 1024" --valu-key scene0_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c2.json
step pmc_c4 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 6 --frames 64" --valu-key scene6_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c4.json
step pmc_c5 300 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 8 --width 3840 --height 2160 --frames 64 --spp 8192" --valu-key scene8_3840x2160_f64_d5 --samples 530841600 --traffic-key "" --out gpurun_out/pmc_c5.json
step kstats_s8 200 python tools/kernel_stats.py --scene 8 --frames 64
exit 0
