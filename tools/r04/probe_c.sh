#!/bin/bash
# Round 4, GPU call C: lane padding of the leaf stage (option lane_pad) -- parity, option A/B on
# scenes 8 / 0 / 6, the stats twin with the <= 8-lane execution counts, and the exec-lane
# microbenchmarks behind it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_pad 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 120 --timeout-method thread -rf -k "lane_pad or lane_padding"
step ab_s8 300 python -u tools/option_ab.py --scene 8 --rounds 5 --specs default,lane_pad=9,lane_pad=12,lane_pad=16,lane_pad=64
step ab_s0 300 python -u tools/option_ab.py --scene 0 --rounds 5 --specs default,lane_pad=9,lane_pad=16,lane_pad=64
step ab_s6 300 python -u tools/option_ab.py --scene 6 --rounds 5 --specs default,lane_pad=9,lane_pad=16,lane_pad=64
step stats_s8_p0 200 python -u tools/kernel_stats.py --scene 8 --frames 64
step stats_s8_p9 200 python -u tools/kernel_stats.py --scene 8 --frames 64 --options '{"lane_pad": 9}'
exit 0
