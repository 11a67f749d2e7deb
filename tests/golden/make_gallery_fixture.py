"""Derive the gallery anchor fixture from the reference's published render (TEST INFRASTRUCTURE).

The reference cannot run in this pipeline (no JDK/LWJGL/GL context, SURVEY
§8c), so its only recorded outputs are the PNGs under galleries/.  The Cornell
box (scene 6, `galleries/book3_final(scene6).png`, 600x600, CLI defaults depth
5) converges fast enough that its 60x60-pixel block means are a statistical
fixture for the whole shading path (mixture PDF, light sampling, materials,
box/quad intersection and App. A Q1/Q2 decisions): 10x10x3 numbers, stored as
JSON.  Scenes 0 and 8 have unseeded geometry (Math.random) and are far from
converged in the gallery, so only their global means are recorded, for
information.

Scenes 0 and 8 also carry fixed geometry whose pixels can be compared (masks
from tests/gallery_regions.py, the same code the tests use):
  * scene 0: the open sky above the horizon, whose bytes are exact: the packed
    mask of pixels equal to the sky colour (217, 230, 255) over rows 0-135;
  * scene 0: the three fixed spheres' means of the linearised bytes (pixels whose ray
    meets them above the random small spheres' layer);
  * scene 8: per deterministic region (light quad, glass / metal / blue-fog /
    earth / Perlin spheres) the pixel count and the mean of the linearised
    bytes ((b/255)^2.2, the inverse of Texture.saveAsPNG's gamma), and the
    earth sphere's 8x8-pixel block means (its texture's pattern).

Reads /root/reference (this container only); the output is committed, and the
tests that use it (tests/test_oracle.py::test_gallery_scene6,
tests/test_gallery_anchor.py) never read the reference.
usage: python tests/golden/make_gallery_fixture.py
"""
import base64
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "raytracing-book_amd")]
import gallery_regions as gr  # noqa: E402
import rtamd  # noqa: E402

SKY_RGB = (217, 230, 255)
SKY_ROWS = 136
EARTH_BLOCK = 8
GALLERY = "/root/reference/galleries"
BLOCK = 60


def block_means(rgb, block):
    h, w = rgb.shape[:2]
    return rgb[:h // block * block, :w // block * block].reshape(
        h // block, block, w // block, block, 3).mean(axis=(1, 3))


def dx2(lin, m):
    """Mean squared difference of horizontally adjacent pixels, both in the mask, per channel:
    twice the per-pixel noise variance plus the (render-independent) texture gradient -- the
    statistic tools/gallery_spp_probe.py matches to estimate the gallery's sample count."""
    both = m[:, 1:] & m[:, :-1]
    d = lin[:, 1:] - lin[:, :-1]
    return np.round((d[both] ** 2).mean(0), 8).tolist()


def main():
    out = {"source": "galleries/book3_final(scene6).png", "block": BLOCK}
    g = np.asarray(Image.open(os.path.join(GALLERY, "book3_final(scene6).png")).convert("RGB")).astype(np.float64)
    out["width"], out["height"] = g.shape[1], g.shape[0]
    out["scene6_block_means"] = np.round(block_means(g, BLOCK), 3).tolist()
    for sid, fn in [(0, "book1_final(scene0).png"), (8, "book2_final(scene8).png")]:
        g = np.asarray(Image.open(os.path.join(GALLERY, fn)).convert("RGB")).astype(np.float64)
        out[f"scene{sid}_global_mean"] = np.round(g.mean(axis=(0, 1)), 3).tolist()
    # scene 0: the exact sky bytes above the horizon
    g0 = np.asarray(Image.open(os.path.join(GALLERY, "book1_final(scene0).png")).convert("RGB"))
    sky = np.all(g0[:SKY_ROWS] == SKY_RGB, axis=-1)
    out["scene0_sky"] = {"source": "galleries/book1_final(scene0).png", "rgb": list(SKY_RGB), "rows": SKY_ROWS,
                         "width": int(g0.shape[1]),
                         "full_rows": int(next(r for r in range(SKY_ROWS) if not sky[r].all())),
                         "mask_packbits_b64": base64.b64encode(np.packbits(sky.reshape(-1)).tobytes()).decode()}
    # scene 0: the three fixed spheres (linearised byte means)
    lin0 = (g0.astype(np.float64) / 255.0) ** 2.2
    h0, w0 = g0.shape[:2]
    regs0 = gr.scene0_regions(rtamd.Scene(0, w0, h0, seed=1).camera, w0, h0)
    out["scene0_regions"] = {"source": "galleries/book1_final(scene0).png", "width": w0, "height": h0,
                             "regions": {k: {"n_pixels": int(m.sum()), "lin_mean": np.round(lin0[m].mean(0), 6).tolist()}
                                         for k, m in regs0.items()}}
    # scene 8: deterministic regions (linearised byte means) and the earth's block pattern
    g8 = np.asarray(Image.open(os.path.join(GALLERY, "book2_final(scene8).png")).convert("RGB")).astype(np.float64)
    lin = (g8 / 255.0) ** 2.2
    h, w = g8.shape[:2]
    cam = rtamd.Scene(8, w, h, seed=1).camera
    regs = gr.scene8_regions(cam, w, h)
    out["scene8_regions"] = {"source": "galleries/book2_final(scene8).png", "width": w, "height": h,
                             "regions": {k: {"n_pixels": int(m.sum()), "lin_mean": np.round(lin[m].mean(0), 6).tolist(),
                                             "byte_mean": np.round(g8[m].mean(0), 3).tolist(),
                                             "lin_dx2": dx2(lin, m),
                                             "frac_255": np.round((g8[m] == 255).mean(0), 6).tolist(),
                                             "all_255": bool((g8[m] == 255).all())}
                                         for k, m in regs.items()}}
    blocks = gr.block_grid(regs["earth"], EARTH_BLOCK)
    out["scene8_earth_blocks"] = {"block": EARTH_BLOCK, "coords": [list(b) for b in blocks],
                                  "lin_means": np.round(gr.block_means(lin, blocks, EARTH_BLOCK), 6).tolist()}
    with open(os.path.join(HERE, "gallery.json"), "w") as f:
        json.dump(out, f, indent=None)
        f.write("\n")


if __name__ == "__main__":
    main()
