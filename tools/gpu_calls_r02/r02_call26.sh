export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|link walk\|%\|smoke" ; [ $rc -eq 0 ] || exit $rc; }


V=0s1000,0s1000t16,0s1000t24,0s1000t48,0s1000t64
step ab_s8 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 8
step ab_s0 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 0
step ab_s6 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 6

step ab_4k 400 python tools/ab_variants.py --variants $V --width 3840 --height 2160 --frames 64 --rounds 3 --scene 8

exit 0
