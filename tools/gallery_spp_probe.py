"""Estimate the sample count of the reference's scene-8 gallery render.

The gallery (galleries/book2_final(scene8).png, 800x600) records neither spp nor max_depth.
Its pixel noise does: the mean squared difference of horizontally adjacent pixels inside a
region (tests/golden/gallery.json "lin_dx2") is twice the per-pixel variance -- which falls
as 1/spp -- plus the texture gradient, the same in any render.  This renders scene 8 on the
GPU progressively (one accumulation, read back at 16, 32, ..., 4096 spp), and reports per
region: the region-mean ratio to the gallery through the PNG pipeline, our dx2 / the
gallery's, and the saturated-byte fraction, so that the spp whose noise matches the
gallery's can be read off, and the region means compared at that sample count (per-pixel
clipping at 1.0 makes the mean of the bytes depend on spp).
usage: python tools/gallery_spp_probe.py [depth] [seed]
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


def dx2(lin, m):
    both = m[:, 1:] & m[:, :-1]
    d = lin[:, 1:] - lin[:, :-1]
    return (d[both] ** 2).mean(0)


def main():
    depth = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    fx = FIX["scene8_regions"]["regions"]
    sc = rtamd.Scene(8, 800, 600, seed=seed)
    regs = gr.scene8_regions(sc.camera, 800, 600)
    total = 4096
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.upload_scene(sc)
    ctx.set_params(max_depth=depth, spp=total)
    ctx.resize(800, 600)
    rf = rtamd.frame_rand_factors(seed, 0, total)
    done, n = 0, 16
    while n <= total:
        while done < n:
            k = min(n - done, 512)
            ctx.render(done + 1, rf[done:done + k])
            done += k
        img = ctx.read_image()
        t8 = rtamd.tonemap_rgb8(img)
        lin = (t8.astype(np.float64) / 255.0) ** 2.2
        rep = {}
        for r in REGIONS:
            m = regs[r]
            rep[r] = {"mean": np.round(lin[m].mean(0) / np.array(fx[r]["lin_mean"]), 4).tolist(),
                      "dx2": np.round(dx2(lin, m) / np.array(fx[r]["lin_dx2"]), 4).tolist(),
                      "sat": np.round((t8[m] == 255).mean(0), 5).tolist()}
        print(json.dumps({"depth": depth, "seed": seed, "spp": n, "regions": rep}), flush=True)
        n *= 2
    ctx.close()


if __name__ == "__main__":
    main()
