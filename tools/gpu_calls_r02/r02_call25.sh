export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|link walk\|%" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step kstats_s8 300 python tools/kernel_stats.py --scene 8 --frames 64
step kstats_s0 300 python tools/kernel_stats.py --scene 0 --frames 64
step ab_n8 400 python tools/ab_variants.py --variants 0 --rank 0 --world 8 --frames 256 --rounds 4 --scene 8
exit 0
