"""Seed-to-seed spread of scene 8's gallery anchor.

The reference's gallery render of scene 8 (galleries/book2_final(scene8).png, 800x600)
used unseeded geometry: the ground boxes' heights and the 1000-sphere cluster come from
Math.random (Scene.java:288-333).  The anchor test compares the regions whose own
geometry is fixed (tests/gallery_regions.py) -- but what surrounds them (reflections,
indirect light, shadows) changes with the seed.  This renders scene 8 at the gallery's
size and 4096 spp on the GPU for seeds 1..8 at max_depth 5 and 6 and reports, per region
and channel, the ratio of the linearised region mean to the gallery's, and its spread
over the seeds.  usage: python tools/gallery_seed_probe.py [seeds] [depths]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import rtamd  # noqa: E402
import gallery_regions as gr  # noqa: E402

FIX = json.load(open(os.path.join(REPO, "tests", "golden", "gallery.json")))
REGIONS = ("glass", "metal", "blue_fog", "earth", "perlin")


def render(seed, depth, spp=4096):
    sc = rtamd.Scene(8, 800, 600, seed=seed)
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.upload_scene(sc)
    ctx.set_params(max_depth=depth, spp=spp)
    ctx.resize(800, 600)
    rf = rtamd.frame_rand_factors(seed, 0, spp)
    for k in range(0, spp, 512):
        ctx.render(k + 1, rf[k:k + 512])
    img = ctx.read_image()
    ctx.close()
    return sc, img


def main():
    seeds = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4,5,6,7,8").split(",")]
    depths = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "5,6").split(",")]
    fx = FIX["scene8_regions"]["regions"]
    summary = {}
    for depth in depths:
        per_seed = []
        for seed in seeds:
            sc, img = render(seed, depth)
            regs = gr.scene8_regions(sc.camera, 800, 600)
            # "png": our image through the reference's PNG pipeline (Texture.saveAsPNG: unorm8, then
            # the truncating gamma) and linearised like the gallery's bytes -- the like-for-like
            # comparison; "raw": the float image itself (what round 2 compared)
            lin_raw = np.clip(np.nan_to_num(img[..., :3], nan=0.0), 0.0, 1.0)
            lin_png = (rtamd.tonemap_rgb8(img).astype(np.float64) / 255.0) ** 2.2
            rat = {kind: {n: (lin[regs[n]].mean(0) / np.array(fx[n]["lin_mean"])).tolist() for n in REGIONS}
                   for kind, lin in (("png", lin_png), ("raw", lin_raw))}
            per_seed.append(rat)
            print(json.dumps({"max_depth": depth, "seed": seed,
                              "ratios": {k: {n: [round(x, 4) for x in v] for n, v in r.items()}
                                         for k, r in rat.items()}}), flush=True)
        agg = {}
        for kind in ("png", "raw"):
            agg[kind] = {}
            for n in REGIONS:
                a = np.array([r[kind][n] for r in per_seed])   # seeds x 3 channels
                agg[kind][n] = {"mean": np.round(a.mean(0), 4).tolist(), "min": np.round(a.min(0), 4).tolist(),
                                "max": np.round(a.max(0), 4).tolist(), "std": np.round(a.std(0, ddof=1), 4).tolist()}
        summary[depth] = agg
        print(json.dumps({"max_depth": depth, "seeds": seeds, "spread": agg}), flush=True)


if __name__ == "__main__":
    main()
