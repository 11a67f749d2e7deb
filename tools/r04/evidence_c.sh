#!/bin/bash
# Round 4 evidence C: the C2 / C4 VALU counts after the built-in redefinitions (their kernels
# changed with rt_glsl.h) merged into profiles/valu.json, then the C2 / C4 bench lines on them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pmc_c2 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 0 --frames 64 --spp 1024" --valu-key scene0_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c2.json
cp gpurun_out/valu.json gpurun_out/valu_c2.json
step pmc_c4 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 6 --frames 64" --valu-key scene6_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c4.json
python - <<'PY'
import json
v = json.load(open("profiles/valu.json"))
v.update(json.load(open("gpurun_out/valu_c2.json")))
v.update(json.load(open("gpurun_out/valu.json")))
json.dump(v, open("profiles/valu.json", "w"), indent=1, sort_keys=True)
json.dump(v, open("gpurun_out/valu_merged.json", "w"), indent=1, sort_keys=True)
PY
step bench_c2 200 python bench.py --preset c2 --cpu-seconds 30
step bench_c4 200 python bench.py --preset c4 --cpu-seconds 30
exit 0
