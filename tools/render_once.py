"""Minimal profiling target: render one batch of frames through rt.h and exit.
usage: python tools/render_once.py [--scene 8] [--width 1920] [--height 1080] [--frames 64] [--launches 1] [--spp 4096]
       [--bvh reference|sah] [--options JSON]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=8)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--depth", type=int, default=5)
ap.add_argument("--launches", type=int, default=1)
ap.add_argument("--spp", type=int, default=4096, help="sqrt_spp uniform")
ap.add_argument("--bvh", default="reference", choices=["reference", "sah"], help="rt_set_bvh_mode")
ap.add_argument("--options", default="{}", help='JSON rt_debug options, e.g. {"box_vnodes": 0}')
a = ap.parse_args()
scene = rtamd.Scene(a.scene, a.width, a.height, seed=1)
import json  # noqa: E402
ctx = rtamd.RenderContext(devices=(0,), options=json.loads(a.options))
ctx.set_bvh_mode(a.bvh)
ctx.upload_scene(scene)
ctx.set_params(max_depth=a.depth, spp=a.spp)
ctx.resize(a.width, a.height)
f = 1
for _ in range(a.launches):
    ctx.render(f, rtamd.frame_rand_factors(1, f - 1, a.frames))
    f += a.frames
ctx.sync()
print("render_once ok", ctx.last_render_ns() / 1e6, "ms (last call)")
