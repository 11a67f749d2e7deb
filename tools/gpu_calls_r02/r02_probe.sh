#!/bin/bash
# Round-2 probe on the GPU box: host CPU facts + oracle thread scaling, the VALU
# issue ceiling microkernel, and bench lines for the default launch, direct mode
# (RT_CHUNK_TARGET=0) and configs C2 (scene 0) / C4 (scene 6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
step valu_peak 60 raytracing-book_amd/bin/valu_peak 200000
step cpu_probe 240 python tools/cpu_probe.py --seconds 5
step bench_default 200 python bench.py --no-cpu-baseline
step bench_direct 200 env RT_CHUNK_TARGET=0 python bench.py --no-cpu-baseline
step bench_s0 200 python bench.py --no-cpu-baseline --scene 0 --spp-total 1024
step bench_s6 200 python bench.py --no-cpu-baseline --scene 6 --spp-total 4096
exit 0
