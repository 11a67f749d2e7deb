"""The custom-scene builder (rt_scene.h rts_new ... rts_finish; rtamd.SceneBuilder):
the reference's Scene.java calls one by one.  Host-side, no GPU needed.

* Built call by call as Scene.java writes them, scenes 6, 7 and 9 come out
  byte-identical to the built-in builders (rts_build): SSBOs, textures, camera.
* The boxes' 48-byte records (rt_debug_box_records, what rt_upload_buffer
  stages for the kernel): every Box.java box without rotation (scene 8's 400
  ground boxes) is compact -- its faces rebuilt from corners and normals equal
  the uploaded ones --, a rotated one (scenes 6, 7) is not.
* Errors: bad handles, reference range checks, calls after rts_finish.
"""
import ctypes
import math

import numpy as np
import pytest

import rtamd
from rtamd.scene import MAT_DIELECTRIC, SceneBuilder

RAD = lambda deg: float(np.float32(math.radians(deg)))  # noqa: E731  (float)Math.toRadians(deg)


def same_scene(a, b):
    for k in range(6):
        assert a.buffers[k] == b.buffers[k], f"binding {k} differs"
    assert len(a.textures) == len(b.textures)
    for ta, tb in zip(a.textures, b.textures):
        assert (ta.slot, ta.format, ta.width, ta.height, ta.data) == (tb.slot, tb.format, tb.width, tb.height, tb.data)
    assert np.array_equal(a.camera.view(np.uint32), b.camera.view(np.uint32))
    assert np.array_equal(a.background, b.background)


def cornell_walls(b, light_emit):
    red = b.lambertian(b.solid(0.65, 0.05, 0.05))
    white = b.lambertian(b.solid(0.73, 0.73, 0.73))
    green = b.lambertian(b.solid(0.12, 0.45, 0.15))
    light = b.diffuse_light(*light_emit)
    return red, white, green, light


def build_scene6(w, h):
    """Scene.java:212-249 (cornellBox) through the builder calls."""
    b = SceneBuilder(seed=1)
    red, white, green, light = cornell_walls(b, (15, 15, 15))
    light_quad = b.quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light)
    b.add(b.quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green))
    b.add(b.quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red))
    b.add(light_quad)
    b.add_light(light_quad)
    b.add(b.quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white))
    b.add(b.quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white))
    b.add(b.quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white))
    box1 = b.box((0, 0, 0), (165, 330, 165), white, translation=(265, 0, 295), rotation=(0, RAD(15), 0))
    glass_sphere = b.sphere((190, 90, 190), 90, b.dielectric(1.5))
    b.add(box1)
    b.add(glass_sphere)
    b.add_light(glass_sphere)
    b.camera(look_from=(278, 278, -800), look_at=(278, 278, 0), vfov=40, background=(0, 0, 0))
    return b.finish(w, h)


def build_scene7(w, h):
    """Scene.java:251-280 (cornellSmoke)."""
    b = SceneBuilder(seed=1)
    red, white, green, light = cornell_walls(b, (7, 7, 7))
    b.add(b.quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green))
    b.add(b.quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red))
    b.add(b.quad((113, 554, 127), (330, 0, 0), (0, 0, 305), light))
    b.add(b.quad((0, 555, 0), (555, 0, 0), (0, 0, 555), white))
    b.add(b.quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white))
    b.add(b.quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white))
    box1 = b.box((0, 0, 0), (165, 330, 165), white, translation=(265, 0, 295), rotation=(0, RAD(15), 0))
    box2 = b.box((0, 0, 0), (165, 165, 165), white, translation=(130, 0, 65), rotation=(0, RAD(-18), 0))
    b.add(b.constant_medium(box1, 0.01, b.isotropic(b.solid(0, 0, 0))))
    b.add(b.constant_medium(box2, 0.01, b.isotropic(b.solid(1, 1, 1))))
    b.camera(look_from=(278, 278, -800), look_at=(278, 278, 0), vfov=40, background=(0, 0, 0))
    return b.finish(w, h)


def build_scene9(w, h):
    """The build-defined Book-1 three spheres."""
    b = SceneBuilder(seed=1)
    b.add(b.sphere((0, -100.5, -1), 100, b.lambertian(b.solid(0.8, 0.8, 0.0))))
    b.add(b.sphere((0, 0, -1.2), 0.5, b.lambertian(b.solid(0.1, 0.2, 0.5))))
    b.add(b.sphere((-1, 0, -1), 0.5, b.dielectric(1.5)))
    b.add(b.sphere((1, 0, -1), 0.5, b.metal(b.solid(0.8, 0.6, 0.2), 0.999)))
    b.camera(look_from=(-2, 2, 1), look_at=(0, 0, -1), vfov=20, defocus_angle=10.0, focus_dist=3.4,
             background=(0.70, 0.80, 1.00))
    return b.finish(w, h)


@pytest.mark.parametrize("sid,fn", [(6, build_scene6), (7, build_scene7), (9, build_scene9)])
def test_builder_reproduces_builtin_scene(sid, fn):
    same_scene(fn(96, 64), rtamd.Scene(sid, 96, 64, seed=1))


def box_records(scene):
    L = rtamd.amd()
    b = scene.buffers[4]
    n = ctypes.c_int()
    nb = len(b) // 480
    out = np.zeros((max(nb, 1), 3, 4), np.float32)
    assert L.rt_debug_box_records(ctypes.create_string_buffer(b, len(b)), len(b), out.ctypes.data, out.nbytes,
                                  ctypes.byref(n)) == 0
    return out[:nb], n.value


@pytest.mark.parametrize("sid,n_boxes,n_compact", [(8, 400, 400), (6, 1, 0), (7, 2, 0)])
def test_box_records(sid, n_boxes, n_compact):
    s = rtamd.Scene(sid, 32, 32, seed=1)
    recs, n = box_records(s)
    assert len(recs) == n_boxes and n == n_compact
    assert (recs[:, 2, 1] == 1.0).sum() == n_compact
    q = np.frombuffer(s.buffers[4], np.float32).reshape(n_boxes, 6, 20)   # 6 quads of 80 B per box
    corners = q[:, :, 4:7]                                                  # each face's q
    for k in range(n_boxes):
        r = recs[k]
        lo = np.array([r[0, 0], r[0, 1], r[0, 2]])
        hi = np.array([r[0, 3], r[1, 0], r[1, 1]])
        assert np.all(lo <= corners[k].min(axis=0) + 1e-3) and np.all(hi >= corners[k].max(axis=0) - 1e-3)
    if n_compact:
        # scene 8's boxes: corners (x0, 0, z0)-(x0 + 100, y1, z0 + 100); normals c * (1 / |c|) are
        # within an ulp of 1 (JOML normalize), not always 1: the record carries them
        assert np.all(np.abs(recs[:, 1, 2:] - 1.0) <= 6e-8) and np.all(np.abs(recs[:, 2, 0] - 1.0) <= 6e-8)
        assert np.any(recs[:, 1, 2:] != 1.0)
        assert np.all(recs[:, 0, 1] == 0.0) and np.all(recs[:, 0, 3] - recs[:, 0, 0] == 100.0)


def test_box_record_rejects_a_face_that_does_not_match():
    s = rtamd.Scene(8, 32, 32, seed=1)
    raw = bytearray(s.buffers[4])
    q = np.frombuffer(raw, np.float32).reshape(400, 6, 20)
    q[3, 2, 8] += np.float32(0.5)   # box 3, face 2: its u.x (no longer -DX)
    s.buffers[4] = bytes(raw)
    recs, n = box_records(s)
    assert n == 399 and recs[3, 2, 1] == 0.0


def test_builder_errors():
    b = SceneBuilder(seed=1)
    white = b.lambertian(b.solid(1, 1, 1))
    with pytest.raises(ValueError, match="material"):
        b.sphere((0, 0, 0), 1.0, 99)
    with pytest.raises(ValueError, match="IOR"):
        b.material(MAT_DIELECTRIC, 0, 3.0)
    with pytest.raises(ValueError, match="Fuzz"):
        b.metal(b.solid(1, 1, 1), 1.0)
    with pytest.raises(ValueError, match="model"):
        b.add(12345)
    q = b.quad((0, 0, 0), (1, 0, 0), (0, 1, 0), white)
    with pytest.raises(ValueError, match="medium"):
        b.constant_medium(b.constant_medium(q, 0.1, white), 0.1, white)
    with pytest.raises(ValueError, match="translation and rotation"):
        b.box((0, 0, 0), (1, 1, 1), white, translation=(1, 0, 0))
    b.add(q)
    s = b.finish(8, 8)
    # the inner ConstantMedium's constructor registered q already (ConstantMedium.java:18), as in Java
    assert s.info["n_quads"] == 2 and s.info["n_bvh_nodes"] == 1
    with pytest.raises(ValueError, match="finished"):
        b.solid(1, 1, 1)


# --- host logic of the round-3 kernel forms (no GPU) -------------------------------------------

def _perlin_texture(sid):
    s = rtamd.Scene(sid, 32, 24, seed=1)
    t = next(t for t in s.textures if t.format == rtamd.scene.TEX_R32F and t.width == 6)
    return np.frombuffer(t.data, dtype=np.float32).copy()


@pytest.mark.parametrize("sid", [3, 5, 8])
def test_perlin_table_packs_exactly(sid):
    """rt_debug_perlin_pack (what rt_upload_texture keeps beside the texture and the kernel's
    perlin_noise_pk reads): row r = (ranvec x, y, z of row r, perm x | perm y << 8 | perm z << 16),
    so every value the reference's noise reads (texture.glsl:38-77: texelFetch, then int() of
    the perm columns) is there unchanged."""
    L = rtamd.amd()
    tex = _perlin_texture(sid)
    out = np.zeros((256, 4), np.float32)
    assert L.rt_debug_perlin_pack(tex.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 6, 256,
                                  out.ctypes.data, out.nbytes) == 1
    t = tex.reshape(256, 6)
    assert np.array_equal(out[:, :3].view(np.uint32), t[:, :3].view(np.uint32))
    packed = out[:, 3].view(np.uint32)
    for k in range(3):
        assert np.array_equal((packed >> (8 * k)) & 0xFF, t[:, 3 + k].astype(np.int64))
    assert np.all(packed >> 24 == 0)


def test_perlin_table_that_does_not_pack_is_refused():
    """A perm entry that is not a whole number 0..255 (or another shape) keeps the texture path."""
    L = rtamd.amd()
    fp = ctypes.POINTER(ctypes.c_float)
    for bad in (3.5, -1.0, 256.0, float("nan")):
        tex = _perlin_texture(8)
        tex.reshape(256, 6)[17, 4] = bad
        assert L.rt_debug_perlin_pack(tex.ctypes.data_as(fp), 6, 256, None, 0) == 0, bad
    tex = _perlin_texture(8)
    assert L.rt_debug_perlin_pack(tex.ctypes.data_as(fp), 6, 128, None, 0) == 0
    assert L.rt_debug_perlin_pack(tex.ctypes.data_as(fp), 3, 512, None, 0) == 0


@pytest.mark.parametrize("sid,lo,hi", [(0, 800, 1000), (1, 1000, 1000), (9, 1000, 1000), (5, 500, 500),
                                       (8, 300, 499), (6, 0, 0), (2, 0, 0)])
def test_sphere_pair_leaf_share(sid, lo, hi):
    """The sphere-pair kernels' criterion (rt_render: >= 500 per mille of the leaves hold two
    spheres, and the boxes not all canonical): scene 0's 485 spheres pair up (898), scenes 1, 3
    and 9 are all sphere pairs, scene 5 exactly half; scene 8's cluster is 400 of its 1000
    leaves (the ground boxes are the rest), the Cornell box has no sphere."""
    L = rtamd.amd()
    bvh = rtamd.Scene(sid, 32, 24, seed=1).buffers[1]
    pm = ctypes.c_int(-1)
    assert L.rt_debug_sphere_pair_leaves(ctypes.create_string_buffer(bvh, len(bvh)), len(bvh), ctypes.byref(pm)) == 0
    assert lo <= pm.value <= hi, pm.value
