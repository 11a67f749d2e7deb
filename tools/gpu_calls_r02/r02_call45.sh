export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|identical\|passed\|failed\|Error\|error\|shape" ; [ $rc -eq 0 ] || exit $rc; }
RT_LOG_SHAPE=1 step ab_s8 300 python tools/ab_variants.py --variants 0,0g0 --frames 64 --rounds 7 --scene 8
step ab_s7 300 python tools/ab_variants.py --variants 0,0g0 --frames 64 --rounds 3 --scene 7
step ab_s2 300 python tools/ab_variants.py --variants 0,0g0 --frames 64 --rounds 3 --scene 2
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
exit 0
