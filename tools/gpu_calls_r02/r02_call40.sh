export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "^raw" "gpurun_out/$name.log" | grep "median\|DIFFER\|passed\|failed\|Error\|error\|Msamples" ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_c3 300 python bench.py --no-cpu-baseline
exit 0
