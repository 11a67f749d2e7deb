export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/pmc_profile.py --groups 14,15 --target "--scene 8 --frames 16" --traffic-key "" --out gpurun_out/pmc_ic_s8.json > gpurun_out/pmc_ic_s8.log 2>&1; echo rc=$?
timeout -k 10 300 python tools/pmc_profile.py --groups 14,15 --target "--scene 0 --frames 16" --traffic-key "" --out gpurun_out/pmc_ic_s0.json > gpurun_out/pmc_ic_s0.log 2>&1; echo rc=$?
