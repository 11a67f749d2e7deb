export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_variants.py --variants 0,40,41,42 --rounds 6 --scene 8 > gpurun_out/ab1_s8.log 2>&1; rc=$?; cat gpurun_out/ab1_s8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_variants.py --variants 0,40,41,42 --rounds 6 --scene 0 > gpurun_out/ab1_s0.log 2>&1; rc=$?; cat gpurun_out/ab1_s0.log; exit $rc
