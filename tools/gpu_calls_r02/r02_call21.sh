export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp profiles/valu.json gpurun_out/valu.json
step pmc_c3 600 python tools/pmc_profile.py --groups 0,2,3,4,15 --target "--scene 8 --frames 64" --valu-key scene8_1920x1080_f64_d5 --traffic-key "" --out gpurun_out/pmc_c3.json
exit 0
