export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
step cur_n8 300 python tools/ab_variants.py --variants 0 --rank 0 --world 8 --frames 512 --rounds 4 --scene 8
step prev_n8 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --rank 0 --world 8 --frames 512 --rounds 4 --scene 8
step cur_n4 300 python tools/ab_variants.py --variants 0 --rank 0 --world 4 --frames 256 --rounds 4 --scene 8
step prev_n4 300 bash tools/ab_swap.sh prev python tools/ab_variants.py --variants 0 --rank 0 --world 4 --frames 256 --rounds 4 --scene 8
step cur_n1 300 python tools/ab_variants.py --variants 0 --frames 64 --rounds 4 --scene 8
exit 0
