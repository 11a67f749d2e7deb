export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/kernel_stats.py --scene 8 --frames 16 > gpurun_out/kstats_s8.log 2>&1; rc=$?; cat gpurun_out/kstats_s8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kernel_stats.py --scene 0 --frames 16 > gpurun_out/kstats_s0.log 2>&1; rc=$?; cat gpurun_out/kstats_s0.log; exit $rc
