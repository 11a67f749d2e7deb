#!/bin/bash
# Round 4 evidence F (the shipped state with the walk + leaf rounds at wave priority 1): the GPU
# suite, smoke, the same-box A/B against no s_setprio (lib/prev) and the two-site form of call AF
# (lib/v_both_prev), the bench lines C3 (with the CPU baseline) / C2 / C4 / C5 and rocprof of C3.
# The VALU counts of evidence E stand: s_setprio adds no vector instruction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep "median\|DIFFER\|passed\|smoke ok" "gpurun_out/$name.log" | cut -c1-200; tail -1 "gpurun_out/$name.log" | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
L=raytracing-book_amd/lib
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step prio_ab4 800 python -u tools/lib_ab.py --libs $L/librtamd.so,$L/prev/librtamd.so,$L/v_both_prev/librtamd.so --scenes 8,0,6,7 --rounds 7
step bench_c3 300 python bench.py
step bench_c2 200 python bench.py --preset c2 --cpu-seconds 30
step bench_c4 200 python bench.py --preset c4 --cpu-seconds 30
step bench_c5 200 python bench.py --preset c5 --no-cpu-baseline --steps 4
step rocprof_c3 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
exit 0
