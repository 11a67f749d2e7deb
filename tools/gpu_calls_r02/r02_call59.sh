export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/gallery_depth_probe.py 5,8,10,20,50 > gpurun_out/gallery_depth.log 2>&1; rc=$?; grep max_depth gpurun_out/gallery_depth.log; exit $rc
