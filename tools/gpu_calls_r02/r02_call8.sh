export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | tail -9; [ $rc -eq 0 ] || exit $rc; }
step ab_s8 300 python tools/ab_variants.py --variants 0w1,0w0 --rounds 6 --scene 8
step kstats_s8 300 python tools/kernel_stats.py --scene 8 --frames 16
exit 0
