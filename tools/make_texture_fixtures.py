#!/usr/bin/env python3
"""Writes the image-texture fixtures of tests/test_gpu_image_textures.py (run in the dev container,
which has Pillow; the GPU box reads the committed files):
  tests/golden/tex_rgba.png        24 x 12 RGBA8, seeded noise over a gradient (GL_RGBA upload)
  tests/golden/tex_progressive.jpg 40 x 20 progressive 4:2:0 JPEG (fancy-upsampled chroma, RGB8)
and, beside each, the bytes rts_decode_image must give (Pillow's decode): *.rgb8 / *.rgba8.
usage: python tools/make_texture_fixtures.py"""
import os

import numpy as np
from PIL import Image

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def main():
    rng = np.random.default_rng(20261018)
    yy, xx = np.mgrid[0:12, 0:24]
    rgba = np.stack([xx * 10, yy * 20, (xx + yy) * 7, 255 - yy * 9], -1) + rng.integers(0, 30, (12, 24, 4))
    Image.fromarray(np.clip(rgba, 0, 255).astype(np.uint8), "RGBA").save(os.path.join(OUT, "tex_rgba.png"))
    yy, xx = np.mgrid[0:20, 0:40]
    rgb = np.stack([xx * 6, 255 - yy * 12, (xx * yy) % 256], -1) + rng.integers(0, 40, (20, 40, 3))
    Image.fromarray(np.clip(rgb, 0, 255).astype(np.uint8), "RGB").save(
        os.path.join(OUT, "tex_progressive.jpg"), quality=80, subsampling=2, progressive=True)
    for name, mode in (("tex_rgba.png", "RGBA"), ("tex_progressive.jpg", "RGB")):
        px = np.asarray(Image.open(os.path.join(OUT, name)).convert(mode))
        px.tofile(os.path.join(OUT, name.rsplit(".", 1)[0] + (".rgba8" if mode == "RGBA" else ".rgb8")))
        print("wrote", name, px.shape)


if __name__ == "__main__":
    main()
