#!/bin/bash
# Round-2 evidence run: GPU tests, PMC (VALU, lanes, DRAM) per config, bench lines for
# C2-C5 (C3 with the CPU baseline) with this run's VALU counts, rocprofv3 kernel stats
# of the C3 bench, the stats build's region timers, and the N-rank rehearsal on one GPU
# (gloo).  Every step has its own limit; a failure stops it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
if [ -z "$SKIP_TESTS" ]; then step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread; fi
step pmc_c3 600 python tools/pmc_profile.py --groups 0,2,3,4,15 --target "--scene 8 --frames 64" --valu-key scene8_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c3.json
step pmc_c2 600 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 0 --frames 64 --spp 1024" --valu-key scene0_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c2.json
step pmc_c4 600 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 6 --frames 64" --valu-key scene6_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c4.json
step pmc_c5 600 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 8 --width 3840 --height 2160 --frames 64 --spp 8192" --valu-key scene8_3840x2160_f64_d5 --samples 530841600 --traffic-key "" --out gpurun_out/pmc_c5.json
# the bench's roofline reads profiles/valu.json: this run's counts
cp gpurun_out/valu.json profiles/valu.json
step bench_c3 400 python bench.py
step bench_c2 300 python bench.py --preset c2 --cpu-seconds 30
step bench_c4 300 python bench.py --preset c4 --cpu-seconds 30
step bench_c5 300 python bench.py --preset c5 --no-cpu-baseline --steps 4
step rocprof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline
step kstats_s8 300 python tools/kernel_stats.py --scene 8 --frames 64
step kstats_s0 300 python tools/kernel_stats.py --scene 0 --frames 64
step kstats_s6 300 python tools/kernel_stats.py --scene 6 --frames 64
step rehearse 600 bash tools/gpu_bench_multi.sh
exit 0
