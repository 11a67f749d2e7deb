export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-1500 ; [ $rc -eq 0 ] || exit $rc; }
step rehearse 600 bash tools/gpu_bench_multi.sh
exit 0
