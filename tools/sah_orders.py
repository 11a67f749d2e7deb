#!/usr/bin/env python3
"""The SAH fast mode's build choices (row f3), measured on CPU with the oracle's counters:
child order (0 larger-first, 2 camera-nearer-first) x SAH prim cost, against the reference BVH.
`est` = 14.7 cycles per node visit + 139 per solid / medium test (the round-4 stats twin's
per-lane costs on scene 8).  Output: profiles/r05_sah_orders.log.

    python tools/sah_orders.py [scenes=8,0] [W H frames]
"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytracing-book_amd"), os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402
import rtamd  # noqa: E402


def view(sc, bvh):
    v = types.SimpleNamespace(**{k: getattr(sc, k) for k in ("textures", "camera", "background", "width", "height")})
    v.buffers = dict(sc.buffers)
    v.buffers[1] = bvh
    return v


def main():
    scenes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,0").split(",")]
    W, H, F = (int(x) for x in (sys.argv[2:5] if len(sys.argv) > 4 else (240, 135, 8)))
    for sid in scenes:
        sc = rtamd.Scene(sid, W, H, seed=1)
        rf = rtamd.frame_rand_factors(1, 0, F)
        rows = [("reference", None, None, sc.buffers[1])]
        for o in (0, 2):
            for kp in (1.0, 2.0, 4.0, 8.0):
                rows.append((f"sah order {o}", o, kp, rtamd.sah_bvh(sc, o, prim_cost=kp)))
        for name, o, kp, bvh in rows:
            img, c = pyoracle.render(pyoracle.OracleScene(view(sc, bvh), max_depth=5, spp=4096), rf, nthreads=8,
                                     counters=True)
            n = c["samples"]
            b = np.frombuffer(bvh, np.int32).reshape(-1, 8)
            lv = [(lo, r) for lo, r in zip(b[:, 6], b[:, 7]) if (lo & 0xFFFF) != 0]
            solid_sph = c["sphere_tests"] / n - 2 * c["medium_tests"] / n   # a medium test = 2 boundary tests
            tests = solid_sph + (c["box_tests"] + c["quad_tests"] + c["medium_tests"]) / n
            est = 14.7 * c["node_visits"] / n + 139 * tests
            print(f"scene {sid} {W}x{H}x{F} {name:12s} cost {kp or 0:3.0f} nodes {len(b):5d} pair leaves "
                  f"{sum(1 for lo, r in lv if lo != r):4d} visits/sample {c['node_visits'] / n:6.2f} solid sph "
                  f"{solid_sph:.2f} box {c['box_tests'] / n:.2f} quad {c['quad_tests'] / n:.2f} medium "
                  f"{c['medium_tests'] / n:.2f} est {est:5.0f} mean {np.nanmean(img[..., :3]):.4f}", flush=True)


if __name__ == "__main__":
    main()
