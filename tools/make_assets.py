"""Decode the reference's texture asset into a dependency-free PPM.

The reference loads src/main/resources/textures/earthmap.jpg through
javax.imageio (ImageTexture.java:22-92).  Since round 6 the scene builder decodes
assets/earthmap.jpg itself (host/image_decode.cpp, the IJG decoder's islow IDCT,
fancy upsampling and YCbCr tables); this script's output, assets/earthmap.ppm
(Pillow's libjpeg-turbo decode, top row first, unshifted), is the pin that decode
is checked against byte for byte (tests/test_image_decode.py).
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
