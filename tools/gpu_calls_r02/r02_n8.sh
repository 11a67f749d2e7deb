export TMPDIR=/tmp; mkdir -p gpurun_out
# one rank's share of an 8-GPU run (rank 0 of 8, 8-row stripes), 256 frames per launch, by work split
timeout -k 10 400 python tools/ab_variants.py --variants 0c0,0c8,0c16,0c32,0c64,0c128 --rank 0 --world 8 --frames 256 --rounds 4 --scene 8 > gpurun_out/ab_n8.log 2>&1; rc=$?; cat gpurun_out/ab_n8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_variants.py --variants 0c0,0c8,0c16,0c32,0c64 --frames 64 --rounds 4 --scene 8 > gpurun_out/ab_n1.log 2>&1; rc=$?; cat gpurun_out/ab_n1.log; exit $rc
