export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|identical\|passed\|failed\|Error\|error\|lds" ; [ $rc -eq 0 ] || exit $rc; }
RT_LOG_SHAPE=1 step cur_s8 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 1 --scene 8
step cur_s8 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene 8
step prev_s8 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene 8
step cur2_s8 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene 8
step prev2_s8 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene 8
step kstats_s8 300 python tools/kernel_stats.py --scene 8 --frames 64
exit 0
