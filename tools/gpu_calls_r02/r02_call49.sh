export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -30 "gpurun_out/$name.log" | grep -i "icache\|SQ_\|error"; [ $rc -eq 0 ] || exit $rc; }
step pmc_ic 300 python tools/pmc_profile.py --groups 14 --target "--scene 8 --frames 64" --valu-key "" --traffic-key "" --out gpurun_out/pmc_ic.json
exit 0
