export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed" ; [ $rc -eq 0 ] || exit $rc; }

step ab_n8r0 400 python tools/ab_variants.py --variants 0,0c8,0c64,0c4s0 --rank 0 --world 8 --frames 256 --rounds 5 --scene 8
step ab_n8r5 400 python tools/ab_variants.py --variants 0,0c8 --rank 5 --world 8 --frames 256 --rounds 5 --scene 8
step ab_4k 400 python tools/ab_variants.py --variants 0,0c0,0s1000 --width 3840 --height 2160 --frames 64 --rounds 4 --scene 8
step ab_4k_n8 400 python tools/ab_variants.py --variants 0,0c8 --width 3840 --height 2160 --rank 0 --world 8 --frames 256 --rounds 4 --scene 8
exit 0
