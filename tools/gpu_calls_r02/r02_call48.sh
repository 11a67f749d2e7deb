export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|identical\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
step ab_s8 300 python tools/ab_variants.py --variants 0,0e0 --frames 64 --rounds 5 --scene 8
step prev_s8 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --frames 64 --rounds 5 --scene 8
exit 0
