export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300 ; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --no-cpu-baseline
exit 0
