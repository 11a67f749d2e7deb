export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ab_n8 400 python tools/ab_variants.py --variants 0,0s0,0c64,0c16 --rank 0 --world 8 --frames 256 --rounds 4 --scene 8
step ab_n2 400 python tools/ab_variants.py --variants 0,0s0 --rank 0 --world 2 --frames 128 --rounds 4 --scene 8
step ab_n1 400 python tools/ab_variants.py --variants 0,0s1000,0c16 --frames 64 --rounds 5 --scene 8
exit 0
