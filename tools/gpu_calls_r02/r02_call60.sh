export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/gallery_depth_probe.py 6,7 > gpurun_out/gallery_depth67.log 2>&1; rc=$?; grep max_depth gpurun_out/gallery_depth67.log; exit $rc
