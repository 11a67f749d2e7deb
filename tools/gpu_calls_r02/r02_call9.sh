export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; echo "list rc=$?"
timeout -k 10 120 env RT_LOG_SHAPE=1 python tools/render_once.py --scene 8 --frames 16 > gpurun_out/shape.log 2>&1; echo "shape rc=$?"; tail -3 gpurun_out/shape.log
