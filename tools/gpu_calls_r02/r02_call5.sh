# GPU tests, bench lines for C2/C3/C4 (+ CPU baseline on C3), PMC for the roofline records
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c3 400 python bench.py
step bench_c2 200 python bench.py --preset c2 --no-cpu-baseline
step bench_c4 200 python bench.py --preset c4 --no-cpu-baseline
step pmc_c3 600 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 8 --frames 64" --valu-key scene8_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c3.json
step pmc_c2 600 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 0 --frames 64 --spp 1024" --valu-key scene0_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c2.json
step pmc_c4 600 python tools/pmc_profile.py --groups 0,2,3,4 --target "--scene 6 --frames 64" --valu-key scene6_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c4.json
exit 0
