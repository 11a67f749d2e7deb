"""Count the algorithmic (logical record) bytes per sample of a bench config with the
oracle's instrumented mode and record them in bench/bytes_per_sample.json.

Counted: framebuffer 32 B (load+store), 32 B per BVH node popped, the record size
per primitive test (sphere 48, quad 80, box 480, medium 20 + boundary), the record
re-read per closer hit, texel bytes per lookup, light records.  Deterministic for
(scene, seed, W, H, frames, depth); the whole image is counted.
usage: python tools/count_bytes.py [--scene 8 --width 1920 --height 1080 --frames 8 --depth 5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

KEYS = ["framebuffer_bytes", "node_bytes", "prim_bytes", "material_bytes", "texel_bytes", "light_bytes"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", type=int, default=8)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--frames", type=int, default=8)
    p.add_argument("--depth", type=int, default=5)
    p.add_argument("--spp-total", type=int, default=4096)
    p.add_argument("--seed", type=int, default=1)
    a = p.parse_args()
    sc = rtamd.Scene(a.scene, a.width, a.height, seed=a.seed)
    o = pyoracle.OracleScene(sc, max_depth=a.depth, spp=a.spp_total)
    t = time.time()
    _, cnt = pyoracle.render(o, rtamd.frame_rand_factors(a.seed, 0, a.frames), counters=True)
    dt = time.time() - t
    n = cnt["samples"]
    rec = {k: cnt[k] / n for k in KEYS + ["bounces", "node_visits", "sphere_tests", "quad_tests", "box_tests",
                                           "medium_tests", "rand_calls"]}
    rec["bytes_per_sample"] = sum(cnt[k] for k in KEYS) / n
    rec["samples_counted"] = n
    rec["config"] = vars(a)
    path = os.path.join(REPO, "bench", "bytes_per_sample.json")
    db = {}
    if os.path.exists(path):
        with open(path) as f:
            db = json.load(f)
    db[f"scene{a.scene}_depth{a.depth}"] = rec
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
    print(f"{n} samples counted in {dt:.1f}s: {rec['bytes_per_sample']:.1f} B/sample")


if __name__ == "__main__":
    main()
