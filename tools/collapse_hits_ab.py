#!/usr/bin/env python3
"""The collapse planned from the walks' own node hits against the camera-ray grid (VERDICT r5 Next 4).

1. Calibration: the stats twin (A/B library) renders `--cal-frames` frames of the scene with the
   collapse and the spine entry off (the rebuilt tree walked whole, every walk from the root) and
   counts, per link node, the box tests that hit, and the walks (rt_debug_count_node_hits).
2. Plans: context G plans the collapse from the camera grid (the default); context M from the
   measured hits (rt_debug_set_collapse_hits).  Both are exact, so their images must be identical.
3. Node lane-steps per sample of both (stats twin, `--stat-frames` frames), then interleaved HIP-event
   timings of the release structure (variant 0) over `--frames` frames.
usage: python tools/collapse_hits_ab.py [--scene 8] [--cal-frames 4] [--frames 64] [--rounds 7]
"""
import argparse
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "raytracing-book_amd"), os.path.join(REPO, "tools")]
import numpy as np  # noqa: E402
import rtamd  # noqa: E402
from kernel_stats import NAMES  # noqa: E402


def node_steps(ctx, frames, samples):
    L = ctx._L
    assert L.rt_debug_enable_stats(ctx._h, 1) == 0
    ctx.resize(ctx.width, ctx.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, frames))
    ctx.sync()
    buf = (ctypes.c_ulonglong * 128)()
    assert L.rt_debug_read_stats(ctx._h, buf, 128) == 0
    assert L.rt_debug_enable_stats(ctx._h, 0) == 0
    v = {n: buf[i] for i, n in enumerate(NAMES)}
    tot = v["TOTAL"] or 1
    return v["NODE_LN"] / samples, 100.0 * v["NODE_CYC"] / tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cal-frames", type=int, default=4)
    ap.add_argument("--stat-frames", type=int, default=8)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--depth", type=int, default=5)
    a = ap.parse_args()
    scene = rtamd.Scene(a.scene, a.width, a.height, seed=1)

    def ctx(options=None):
        c = rtamd.RenderContext(devices=(0,), ab=True, options=options)
        c.upload_scene(scene)
        c.set_params(max_depth=a.depth, spp=4096)
        c.resize(a.width, a.height)
        return c

    cal = ctx({"collapse": 0, "spine": 0})
    assert cal._L.rt_debug_enable_stats(cal._h, 1) == 0
    cal.count_node_hits(True)
    # calibration frames taken after the timed ones' (frame indices 1000..), so the plan is not fitted
    # to the very samples it is timed on
    cal.render(1000, rtamd.frame_rand_factors(1, 999, a.cal_frames))
    cal.sync()
    hits, walks = cal.read_node_hits()
    print(f"scene {a.scene}: calibration {a.cal_frames} frames, {len(hits)} link nodes, {walks} walks from the root, "
          f"root hits {hits[0]}", flush=True)

    ctxs = {"grid": ctx(), "measured": ctx()}
    ctxs["measured"].set_collapse_hits(hits, walks)
    samples_stat = a.width * a.height * a.stat_frames
    for k, c in ctxs.items():
        steps, share = node_steps(c, a.stat_frames, samples_stat)
        print(f"{k}: node lane-steps per sample {steps:.2f}, node walk {share:.1f}% of wave-cycles; "
              f"launch {c.last_launch()}", flush=True)
    rf = rtamd.frame_rand_factors(1, 0, a.frames)
    times = {k: [] for k in ctxs}
    ref = None
    for r in range(a.rounds + 1):
        for k, c in ctxs.items():
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
                    print(f"{k}: bits {'identical' if same else 'DIFFER'} to grid", flush=True)
                continue
            times[k].append(ns / 1e6)
    samples = a.width * a.height * a.frames
    for k in ctxs:
        med = statistics.median(times[k])
        print(f"scene {a.scene} {k}: median {med:.3f} ms  min {min(times[k]):.3f} ms  -> "
              f"{samples / med / 1e3:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
