export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
V=0,46
step ab_s8 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 4 --scene 8
step ab_s0 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 4 --scene 0
exit 0
