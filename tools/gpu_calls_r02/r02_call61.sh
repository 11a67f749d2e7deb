export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gallery_anchor.py -m gpu -x -v -s --timeout 240 --timeout-method thread -k scene0_fixed > gpurun_out/gallery0_gpu.log 2>&1; rc=$?
grep -i "region mean\|passed\|failed\|Error" gpurun_out/gallery0_gpu.log | cut -c1-400 | head -20; exit $rc
