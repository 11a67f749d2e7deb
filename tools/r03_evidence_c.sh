#!/bin/bash
# Round-3 evidence after the branch-free built-ins (run after r03_evidence_a.sh, whose PMC
# passes are copied into profiles/valu.json first): bench lines C2-C5 (C3 with the 60 s CPU
# baseline), rocprofv3 kernel stats of the C3 bench, the N-rank rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step bench_c3 300 python bench.py
step bench_c2 200 python bench.py --preset c2 --cpu-seconds 30
step bench_c4 200 python bench.py --preset c4 --cpu-seconds 30
step bench_c5 200 python bench.py --preset c5 --no-cpu-baseline --steps 4
step rocprof_c3 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
step rehearse 400 bash tools/gpu_bench_multi.sh
exit 0
