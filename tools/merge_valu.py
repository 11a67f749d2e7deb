#!/usr/bin/env python3
"""Merge the roofline records tools/pmc_profile.py wrote (--valu-out files) into profiles/valu.json,
the file bench.py's roofline reads; writes gpurun_out/valu_merged.json too (the GPU box's copy of
profiles/ is not merged back, gpurun_out/ is).  usage: python tools/merge_valu.py FILE..."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    path = os.path.join(REPO, "profiles", "valu.json")
    v = json.load(open(path)) if os.path.exists(path) else {}
    for f in sys.argv[1:]:
        if os.path.exists(f):
            v.update(json.load(open(f)))
            print("merged", f)
    for p in (path, os.path.join(REPO, "gpurun_out", "valu_merged.json")):
        with open(p, "w") as fh:
            json.dump(v, fh, indent=1, sort_keys=True)
    print(json.dumps({k: (r.get("SQ_INSTS_VALU"), r.get("valu_lane_utilization")) for k, r in v.items()}, indent=1))


if __name__ == "__main__":
    main()
