export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ab_s8 300 python tools/ab_variants.py --variants 0,30 --rounds 6 --scene 8
step ab_s0 300 python tools/ab_variants.py --variants 0,30 --rounds 6 --scene 0
exit 0
