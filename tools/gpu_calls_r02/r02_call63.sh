export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
for sc in 8 0 6; do
step cur_s$sc 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 5 --scene $sc
for t in w1 w3 w4; do
step ${t}_s$sc 300 bash tools/ab_swap.sh $t python tools/ab_variants.py --variants 0 --frames 64 --rounds 5 --scene $sc
done
done
exit 0
