export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_r2a.log 2>&1 && tail -1 gpurun_out/bench_r2a.log
timeout -k 10 200 env RT_CHUNK_TARGET=0 python bench.py --no-cpu-baseline > gpurun_out/bench_r2a_direct.log 2>&1 && tail -1 gpurun_out/bench_r2a_direct.log
