export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gallery_anchor.py -m gpu -x -v -s --timeout 240 --timeout-method thread > gpurun_out/gallery_gpu.log 2>&1; rc=$?
grep -i "ratio\|correlation\|passed\|failed\|Error" gpurun_out/gallery_gpu.log | head -20; exit $rc
