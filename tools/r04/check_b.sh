#!/bin/bash
# Round 4, GPU check B (shading tables in LDS on by default): the GPU suite, smoke, and the C3 / C2 /
# C4 bench lines (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-260; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 200 python bench.py --no-cpu-baseline
step bench_c2 200 python bench.py --preset c2 --no-cpu-baseline
step bench_c4 200 python bench.py --preset c4 --no-cpu-baseline
exit 0
