export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|identical\|passed\|failed\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
for sc in 8 0 6; do
step cur${r}_s$sc 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 5 --scene $sc
step prev${r}_s$sc 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --frames 64 --rounds 5 --scene $sc
done
done
exit 0
