export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -30 "gpurun_out/$name.log" | grep -v "^group\|target" ; [ $rc -eq 0 ] || exit $rc; }
step pmc_mem 600 python tools/pmc_profile.py --groups 0,12,13,5 --target "--scene 8 --frames 64" --traffic-key "" --out gpurun_out/pmc_mem_s8.json
exit 0
