#!/bin/bash
# Round 4, GPU call M: where the two-level kernel's fixed ~10% goes -- the stats twin's region
# breakdown of the 4000-sphere cloud all in LDS, with 31 nodes global (cap 130048 B) and with
# three quarters global (cap 32768 B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; cat "gpurun_out/$name.log" | grep -v "^raw\|amdgpu.ids" | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step kstats_cloud_all 200 python tools/kernel_stats.py --cloud 4000 --frames 16
step kstats_cloud_130k 200 python tools/kernel_stats.py --cloud 4000 --frames 16 --options '{"lds_node_cap": 130048}'
step kstats_cloud_32k 200 python tools/kernel_stats.py --cloud 4000 --frames 16 --options '{"lds_node_cap": 32768}'
exit 0
