#!/bin/bash
# Round 4, GPU call B: per-type leaf deferral (option leaf_defer) -- parity (small vs the oracle,
# full size vs the default), option A/B on scenes 8 / 0 / 6, the stats twin's lane use with and
# without it, and the CPU oracle's thread scaling inside the job's quota.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step pytest_defer 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 120 --timeout-method thread -rf -k "leaf_defer or leaf_deferral"
step ab_s8 300 python -u tools/option_ab.py --scene 8 --rounds 5 --specs default,leaf_defer=8,leaf_defer=16,leaf_defer=24,leaf_defer=32
step ab_s0 300 python -u tools/option_ab.py --scene 0 --rounds 5 --specs default,leaf_defer=8,leaf_defer=16,leaf_defer=24,leaf_defer=32
step ab_s6 300 python -u tools/option_ab.py --scene 6 --rounds 5 --specs default,leaf_defer=8,leaf_defer=16,leaf_defer=24,leaf_defer=32
step stats_s8_d0 200 python -u tools/kernel_stats.py --scene 8 --frames 64
step stats_s8_d16 200 python -u tools/kernel_stats.py --scene 8 --frames 64 --options '{"leaf_defer": 16}'
step cpu_probe 200 python -u tools/cpu_probe.py --seconds 6 --threads 1,4,8,12,14,16
exit 0
