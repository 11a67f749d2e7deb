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

Reads /root/reference (this container only); the output is committed, and the
test that uses it (tests/test_oracle.py::test_gallery_scene6) never reads the
reference.
usage: python tests/golden/make_gallery_fixture.py
"""
import json
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
GALLERY = "/root/reference/galleries"
BLOCK = 60


def block_means(rgb, block):
    h, w = rgb.shape[:2]
    return rgb[:h // block * block, :w // block * block].reshape(
        h // block, block, w // block, block, 3).mean(axis=(1, 3))


def main():
    out = {"source": "galleries/book3_final(scene6).png", "block": BLOCK}
    g = np.asarray(Image.open(os.path.join(GALLERY, "book3_final(scene6).png")).convert("RGB")).astype(np.float64)
    out["width"], out["height"] = g.shape[1], g.shape[0]
    out["scene6_block_means"] = np.round(block_means(g, BLOCK), 3).tolist()
    for sid, fn in [(0, "book1_final(scene0).png"), (8, "book2_final(scene8).png")]:
        g = np.asarray(Image.open(os.path.join(GALLERY, fn)).convert("RGB")).astype(np.float64)
        out[f"scene{sid}_global_mean"] = np.round(g.mean(axis=(0, 1)), 3).tolist()
    with open(os.path.join(HERE, "gallery.json"), "w") as f:
        json.dump(out, f, indent=None)
        f.write("\n")


if __name__ == "__main__":
    main()
