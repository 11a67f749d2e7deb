export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|link walk\|%\|smoke" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ab_n8 400 python tools/ab_variants.py --variants 0,0t32,0t64 --rank 0 --world 8 --frames 256 --rounds 4 --scene 8
step ab_n2 400 python tools/ab_variants.py --variants 0,0t32 --rank 1 --world 2 --frames 128 --rounds 4 --scene 8
step ab_4k_n8 400 python tools/ab_variants.py --variants 0,0t32 --width 3840 --height 2160 --rank 7 --world 8 --frames 256 --rounds 3 --scene 8
step kstats_s8 300 python tools/kernel_stats.py --scene 8 --frames 64
exit 0
