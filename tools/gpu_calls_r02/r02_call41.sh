export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|identical\|passed\|failed\|Error\|error\|LEAF\|leaf-slot\|NODE\|SHADE" ; [ $rc -eq 0 ] || exit $rc; }
step ab_s8 300 python tools/ab_variants.py --variants 0,0l1 --frames 64 --rounds 5 --scene 8
step ab_s0 300 python tools/ab_variants.py --variants 0,0l1 --frames 64 --rounds 5 --scene 0
step ab_s6 300 python tools/ab_variants.py --variants 0,0l1 --frames 64 --rounds 5 --scene 6
RT_LEAF_COMPACT=1 step kstats_s8_l1 300 python tools/kernel_stats.py --scene 8 --frames 64
exit 0
