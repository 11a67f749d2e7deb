export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|link walk\|%" ; [ $rc -eq 0 ] || exit $rc; }
V=0,0c16,0c12,0c8,0c16f52,0c16f48
step ab_s8 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 4 --scene 8
step ab_s0 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 4 --scene 0
step ab_s6 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 4 --scene 6
step ab_4k 400 python tools/ab_variants.py --variants 0,0c16,0c8 --width 3840 --height 2160 --frames 64 --rounds 3 --scene 8
exit 0
