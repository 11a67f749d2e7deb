#!/bin/bash
# Round-3 final evidence, part B: the C2 PMC pass again (its kernel changed after part A: the
# sphere-pair kernels), merged into the profiles/valu.json the bench lines read; bench lines
# C2-C5 (C3 with the 60 s CPU baseline), rocprofv3 kernel stats of the C3 bench, the N-rank
# rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pmc_c2 240 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 0 --frames 64 --spp 1024" --valu-key scene0_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c2.json
python - <<'PY'
import json
v = json.load(open("profiles/valu.json"))
v.update(json.load(open("gpurun_out/valu.json")))
json.dump(v, open("profiles/valu.json", "w"), indent=1, sort_keys=True)
json.dump(v, open("gpurun_out/valu_merged.json", "w"), indent=1, sort_keys=True)
PY
step bench_c3 300 python bench.py
step bench_c2 200 python bench.py --preset c2 --cpu-seconds 30
step bench_c4 200 python bench.py --preset c4 --cpu-seconds 30
step bench_c5 200 python bench.py --preset c5 --no-cpu-baseline --steps 4
step rocprof_c3 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
step rehearse 400 bash tools/gpu_bench_multi.sh
exit 0
