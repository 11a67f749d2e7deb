#!/bin/bash
# Round 4 evidence E (the shipped state: built-in redefinitions, shading tables in LDS, walk thresholds by BVH size): the GPU suite and smoke, the C3 / C5 PMC
# passes merged into profiles/valu.json (the roofline's VALU counts), the bench lines C3 (with the
# CPU baseline on the quota's threads), C2, C4, C5, rocprofv3 kernel stats of the C3 bench and the
# stats twin's region breakdown of scene 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step pmc_c3 300 python tools/pmc_profile.py --groups 0,2,3,4,5,15 --target "--scene 8 --frames 64" --valu-key scene8_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c3.json
cp gpurun_out/valu.json gpurun_out/valu_c3.json
step pmc_c5 300 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 8 --width 3840 --height 2160 --frames 64 --spp 8192" --valu-key scene8_3840x2160_f64_d5 --samples 530841600 --traffic-key "" --out gpurun_out/pmc_c5.json
cp gpurun_out/valu.json gpurun_out/valu_c5.json
step pmc_c2 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 0 --frames 64 --spp 1024" --valu-key scene0_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c2.json
cp gpurun_out/valu.json gpurun_out/valu_c2.json
step pmc_c4 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 6 --frames 64" --valu-key scene6_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c4.json
python - <<'PY'
import json
v = json.load(open("profiles/valu.json"))
for f in ("valu_c3", "valu_c5", "valu_c2", "valu"):
    v.update(json.load(open(f"gpurun_out/{f}.json")))
json.dump(v, open("profiles/valu.json", "w"), indent=1, sort_keys=True)
json.dump(v, open("gpurun_out/valu_merged.json", "w"), indent=1, sort_keys=True)
PY
step bench_c3 300 python bench.py
step bench_c2 200 python bench.py --preset c2 --cpu-seconds 30
step bench_c4 200 python bench.py --preset c4 --cpu-seconds 30
step bench_c5 200 python bench.py --preset c5 --no-cpu-baseline --steps 4
step rocprof_c3 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
step kstats_s8 200 python tools/kernel_stats.py --scene 8 --frames 64
exit 0
