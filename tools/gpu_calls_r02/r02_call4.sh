export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python -c "
import sys,time; sys.path[:0]=['raytracing-book_amd','tests','oracle']
import os; os.environ['RT_CHUNK_TARGET']='100000'
import rtamd, numpy as np
from helpers import gpu_image, oracle_image, bit_equal, mismatch_report
s=rtamd.Scene(6,40,24,seed=1)
t=time.time(); out=gpu_image(s,6); print('gpu s', time.time()-t)
ref=oracle_image(s,6); print('equal', bit_equal(out,ref), mismatch_report(out,ref))
" > gpurun_out/small_chunked.log 2>&1; rc=$?; cat gpurun_out/small_chunked.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_r2a.log 2>&1 && tail -1 gpurun_out/bench_r2a.log
timeout -k 10 200 env RT_CHUNK_TARGET=0 python bench.py --no-cpu-baseline > gpurun_out/bench_r2a_direct.log 2>&1 && tail -1 gpurun_out/bench_r2a_direct.log
