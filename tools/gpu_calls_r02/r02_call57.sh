export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|identical\|passed\|failed\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for sc in 8 6; do
step cur_s$sc 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene $sc
step prev_s$sc 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene $sc
done
step cur2_s8 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene 8
step prev2_s8 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --frames 64 --rounds 7 --scene 8
exit 0
