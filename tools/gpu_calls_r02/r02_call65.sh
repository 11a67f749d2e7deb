export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
V=0,0w40,0w44,0w52,0w56
step wf_s8 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 8
step wf_s0 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 0
step wf_s6 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 6
exit 0
