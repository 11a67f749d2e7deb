"""Decode the reference's texture asset into a dependency-free PPM.

The reference loads src/main/resources/textures/earthmap.jpg through
javax.imageio (ImageTexture.java:22-92).  /root/reference is absent on the GPU
box and the C++ scene builder has no JPEG decoder, so the decoded RGB8 pixels
(top row first, unshifted; ImageTexture's flip/shift is applied by the builder)
are committed as assets/earthmap.ppm.  Decoder: Pillow's libjpeg; Java ImageIO's
IDCT may differ by +-1 per channel (texture bits are not pinned by any test).
Run in the dev container: python tools/make_assets.py
"""
import os
import sys

from PIL import Image

SRC = "/root/reference/src/main/resources/textures/earthmap.jpg"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "assets", "earthmap.ppm")


def main():
    img = Image.open(SRC).convert("RGB")
    w, h = img.size
    with open(DST, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(img.tobytes())
    print("wrote", DST, w, h)


if __name__ == "__main__":
    sys.exit(main())
