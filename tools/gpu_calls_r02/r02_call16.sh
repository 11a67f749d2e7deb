export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|link walk\|%" ; [ $rc -eq 0 ] || exit $rc; }
V=40,0b40,0b48,0b56,0b48f48,0b48f40,0b56f48,0b64f48,0b64f56,0b40f56
step ab_s8 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 3 --scene 8
step ab_s0 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 3 --scene 0
step ab_s6 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 3 --scene 6
exit 0
