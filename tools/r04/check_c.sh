#!/bin/bash
# Round 4, GPU check C (walk_frac by BVH size): the GPU suite, smoke, the new default against the
# old fixed 48 on scenes 6 / 7 / 0 / 8, and the C4 / C2 / C3 bench lines (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|passed\|smoke\|\"value\"" "gpurun_out/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step wf_s6 200 python -u tools/option_ab.py --specs default,walk_frac=48 --scene 6 --rounds 7
step wf_s7 200 python -u tools/option_ab.py --specs default,walk_frac=48 --scene 7 --rounds 7
step wf_s0 200 python -u tools/option_ab.py --specs default,walk_frac=48 --scene 0 --rounds 7
step wf_s8 200 python -u tools/option_ab.py --specs default,walk_frac=48 --scene 8 --rounds 7
step bench_c4 200 python bench.py --preset c4 --no-cpu-baseline
step bench_c2 200 python bench.py --preset c2 --no-cpu-baseline
step bench_c3 200 python bench.py --no-cpu-baseline
exit 0
