export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
V=0,0p0
step ab_s6 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 6
step ab_s7 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 5 --scene 7
step ab_s8 400 python tools/ab_variants.py --variants $V --frames 64 --rounds 3 --scene 8
exit 0
