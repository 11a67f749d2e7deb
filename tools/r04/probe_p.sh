#!/bin/bash
# Round 4, GPU call P: the shading tables in LDS (option shade_lds) -- parity on every scene and
# the adversarial cases with it on, then interleaved A/Bs against the default on scenes 8 / 0 / 6
# at 1080p.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest_sl 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py -m gpu -q -x --timeout 300 --timeout-method thread -k "shading_tables or adversarial_case" -rf
step ab_sl8 300 python -u tools/option_ab.py --specs default,shade_lds=1 --scene 8 --rounds 7
step ab_sl0 300 python -u tools/option_ab.py --specs default,shade_lds=1 --scene 0 --rounds 7
step ab_sl6 300 python -u tools/option_ab.py --specs default,shade_lds=1 --scene 6 --rounds 7
exit 0
