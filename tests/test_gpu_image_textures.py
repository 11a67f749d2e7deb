"""Image textures a host names at run time (ImageTexture.create, ImageTexture.java:22-92), through
the scene builder's decoder (rts_decode_image) into a render, bit for bit against the CPU oracle.

The reference's scenes only texture spheres with one baseline 4:4:4 JPEG (earthmap.jpg, covered by
scenes 2 and 8 everywhere else).  Here a custom scene puts a 4-component PNG (GL_RGBA upload, the
kernel's RGBA8 texel form) on a sphere and a box, and a progressive 4:2:0 JPEG (fancy-upsampled
chroma) on a quad -- the quad's uv (alpha, beta) and the sphere's uv (get_sphere_uv) both sample
them -- under a registered light (mixture PDF) with the walls' solid colours around.
Fixtures: tests/golden/tex_rgba.png, tex_progressive.jpg and their decoded bytes (Pillow's decode,
tools/make_texture_fixtures.py)."""
import os

import numpy as np
import pytest

import rtamd
from helpers import bit_equal, gpu_image, mismatch_report, oracle_image

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_fixtures_decode_to_their_committed_bytes():
    a = rtamd.decode_image(os.path.join(GOLD, "tex_rgba.png"))
    assert a.shape == (12, 24, 4)
    assert np.array_equal(a.ravel(), np.fromfile(os.path.join(GOLD, "tex_rgba.rgba8"), np.uint8))
    b = rtamd.decode_image(os.path.join(GOLD, "tex_progressive.jpg"))
    assert b.shape == (20, 40, 3)
    assert np.array_equal(b.ravel(), np.fromfile(os.path.join(GOLD, "tex_progressive.rgb8"), np.uint8))


def textured_scene(W=64, H=36):
    b = rtamd.SceneBuilder(seed=1)
    rgba = b.image(os.path.join(GOLD, "tex_rgba.png"), 5, 3)
    jpg = b.image(os.path.join(GOLD, "tex_progressive.jpg"), 0, 0)
    white = b.lambertian(b.solid(0.73, 0.73, 0.73))
    b.add(b.sphere((-1.1, 0.2, -4), 0.9, b.lambertian(rgba)))
    b.add(b.box((0.4, -1, -5), (1.6, 0.4, -3.8), b.lambertian(rgba)))
    b.add(b.quad((-3, -1.5, -7), (6, 0, 0), (0, 4, 0), b.lambertian(jpg)))
    b.add(b.quad((-3, -1.5, -7), (0, 0, 7), (6, 0, 0), white))   # floor
    lq = b.add(b.quad((-1, 2.4, -5), (2, 0, 0), (0, 0, 2), b.diffuse_light(8, 8, 8)))
    b.add_light(lq)
    b.camera(look_from=(0, 0.3, 1), look_at=(0, 0, -4), vfov=60, background=(0.1, 0.1, 0.12))
    return b.finish(W, H)


def test_texture_slots_hold_the_decoded_images():
    sc = textured_scene()
    by_size = {(t.width, t.height): t for t in sc.textures}
    t = by_size[(24, 12)]
    assert t.format == rtamd.scene.TEX_RGBA8
    src = np.fromfile(os.path.join(GOLD, "tex_rgba.rgba8"), np.uint8).reshape(12, 24, 4)
    want = np.roll(np.roll(src[::-1], 5, axis=1), 3, axis=0)   # ImageTexture's flip, then the wrap shifts
    assert np.array_equal(np.frombuffer(bytes(t.data), np.uint8).reshape(12, 24, 4), want)
    assert by_size[(40, 20)].format == rtamd.scene.TEX_RGB8


@pytest.mark.gpu
@pytest.mark.parametrize("frames,depth", [(4, 5), (2, 8)])
def test_image_textured_custom_scene_matches_oracle(gpu, frames, depth):
    sc = textured_scene()
    g = gpu_image(sc, frames, max_depth=depth)
    o = oracle_image(sc, frames, max_depth=depth)
    assert bit_equal(g, o), mismatch_report(g, o)
    assert float(np.nanmean(g[..., :3])) > 0.01   # lit, not a black frame
