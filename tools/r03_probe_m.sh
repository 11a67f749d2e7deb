#!/bin/bash
# Round 3, GPU call M: kernel change under test (see the commit) -- the GPU suite, the working
# tree's library against HEAD's on scenes 8 / 0 / 6, and rocprof of the C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf
step lib_ab 400 python -u tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/librtamd_head.so --scenes 8,0,6 --rounds 7
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
exit 0
