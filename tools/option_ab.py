"""Interleaved in-process A/B of the release library's exact options (rt_debug.h RT_OPTION_*).

Each spec is "default" or "name=value[;name=value...]" over rtamd.OPTIONS (options below 100:
layout / exact-form switches, every one bit-identical by contract -- checked here on the
warm-up round).  Timings: HIP-event device time of one rt_render call per round, median and
min over rounds.
usage: python tools/option_ab.py --specs default,spine=0 [--scene 8] [--rounds 7]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
import numpy as np  # noqa: E402
import rtamd  # noqa: E402


def parse(spec):
    if spec == "default":
        return {}
    out = {}
    for kv in spec.split(";"):
        k, v = kv.split("=")
        out[k] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", default="default,spine=0")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--ab", action="store_true", help="the A/B library (ablation options such as debug_flags; "
                                                        "their images are not bit-identical by design)")
    a = ap.parse_args()
    specs = a.specs.split(",")
    scene = rtamd.Scene(a.scene, a.width, a.height, seed=1)
    ctxs = {}
    for s in specs:
        c = rtamd.RenderContext(devices=(0,), options=parse(s), ab=a.ab)
        c.upload_scene(scene)
        c.set_params(max_depth=a.depth, spp=4096)
        c.resize(a.width, a.height)
        ctxs[s] = c
    rf = rtamd.frame_rand_factors(1, 0, a.frames)
    times = {s: [] for s in specs}
    ref = None
    for r in range(a.rounds + 1):
        for s in specs:
            c = ctxs[s]
            c.resize(a.width, a.height)   # zero the image: the same inputs every round
            c.render(1, rf)
            c.sync()
            ns = c.last_render_ns()
            if r == 0:
                img = c.read_image()
                if ref is None:
                    ref = img
                else:
                    same = np.array_equal(img.view(np.uint32), ref.view(np.uint32))
                    print(f"{s}: bits {'identical' if same else 'DIFFER'} to {specs[0]}; launch {c.last_launch()}",
                          flush=True)
                continue
            times[s].append(ns / 1e6)
    samples = a.width * a.height * a.frames
    for s in specs:
        med = statistics.median(times[s])
        print(f"scene {a.scene} {s}: median {med:.3f} ms  min {min(times[s]):.3f} ms  -> "
              f"{samples / med / 1e3:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
