export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|link walk\|%" ; [ $rc -eq 0 ] || exit $rc; }
step ab_n8 400 python tools/ab_variants.py --variants 0,0c16,0c64 --rank 0 --world 8 --frames 256 --rounds 4 --scene 8
step ab_n2 400 python tools/ab_variants.py --variants 0,0c16 --rank 1 --world 2 --frames 128 --rounds 4 --scene 8
step ab_n4 400 python tools/ab_variants.py --variants 0,0c16 --rank 3 --world 4 --frames 256 --rounds 4 --scene 8
step ab_4k_n8 400 python tools/ab_variants.py --variants 0,0c16 --width 3840 --height 2160 --rank 7 --world 8 --frames 256 --rounds 3 --scene 8
exit 0
