"""Interleaved in-process A/B of library builds (the working tree's against a previous
revision's kernel, built by tools/build_prev_lib.sh): the same scene, options and frames on
each, bits compared on the warm-up round, HIP-event device time per rt_render call.
usage: python tools/lib_ab.py --libs raytracing-book_amd/lib/librtamd.so,raytracing-book_amd/lib/prev/librtamd.so
  [--scenes 8,0 | --clouds 4000:4,9000:9] [--options '{"lds_node_cap": 98304}']
(--clouds: tests/adversarial.py sphere_cloud(n, seed), the BVH-size cases of tools/bvh_scaling.py)
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import json  # noqa: E402
import numpy as np  # noqa: E402
import rtamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--scenes", default="8")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--clouds", default="")
    ap.add_argument("--options", default="{}")
    a = ap.parse_args()
    libs = a.libs.split(",")
    opts = json.loads(a.options)
    cases = []
    if a.clouds:
        import adversarial
        for spec in a.clouds.split(","):
            n, seed = (int(x) for x in spec.split(":"))
            cases.append((f"cloud{n}", adversarial.sphere_cloud(n, seed, W=a.width, H=a.height)))
    else:
        cases = [(int(x), rtamd.Scene(int(x), a.width, a.height, seed=1)) for x in a.scenes.split(",")]
    for sid, scene in cases:
        ctxs = []
        for lib in libs:
            c = rtamd.RenderContext(devices=(0,), lib=os.path.join(REPO, lib), options=opts or None)
            c.upload_scene(scene)
            c.set_params(max_depth=a.depth, spp=4096)
            c.resize(a.width, a.height)
            ctxs.append(c)
        rf = rtamd.frame_rand_factors(1, 0, a.frames)
        times = [[] for _ in libs]
        ref = None
        for r in range(a.rounds + 1):
            for k, c in enumerate(ctxs):
                c.resize(a.width, a.height)
                c.render(1, rf)
                c.sync()
                ns = c.last_render_ns()
                if r == 0:
                    img = c.read_image()
                    if ref is None:
                        ref = img
                    else:
                        same = np.array_equal(img.view(np.uint32), ref.view(np.uint32))
                        print(f"scene {sid} {libs[k]}: bits {'identical' if same else 'DIFFER'} to {libs[0]}",
                              flush=True)
                    continue
                times[k].append(ns / 1e6)
        samples = a.width * a.height * a.frames
        for k, lib in enumerate(libs):
            med = statistics.median(times[k])
            print(f"scene {sid} {lib}: median {med:.3f} ms  min {min(times[k]):.3f} ms  -> "
                  f"{samples / med / 1e3:.1f} Msamples/s", flush=True)
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
