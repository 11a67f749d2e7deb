"""CPU tests of the host side: java.util.Random restatement, scene builder, packers, tonemap/PNG.

The scene builder restates J/draw/Scene.java + the model/texture/material
classes (J/models, J/draw/textures, J/draw/Material.java) and packs the SSBOs
the way RaytraceModel.putModelsToProgram does (RaytraceModel.java:139-246).
"""
import math
import struct

import numpy as np
import pytest

import rtamd
from rtamd import scene as S

# --- java.util.Random (JDK 17 published algorithm) ---------------------------------------------

MASK48 = (1 << 48) - 1


class PyJavaRandom:
    """Independent pure-Python restatement of java.util.Random's LCG."""

    def __init__(self, seed):
        self.s = (seed ^ 0x5DEECE66D) & MASK48

    def next(self, bits):
        self.s = (self.s * 0x5DEECE66D + 0xB) & MASK48
        v = self.s >> (48 - bits)
        return v - (1 << bits) if v >= 1 << (bits - 1) else v

    def next_int(self):
        return self.next(32)

    def next_double(self):
        hi = self.next(26) & ((1 << 26) - 1)
        lo = self.next(27) & ((1 << 27) - 1)
        return ((hi << 27) + lo) * 2.0 ** -53

    def next_float(self):
        return (self.next(24) & ((1 << 24) - 1)) / float(1 << 24)


def test_java_random_known_answers():
    L = rtamd.scene_lib()
    # published JDK values: new Random(42).nextInt() x4, new Random(0).nextInt()
    assert [L.rts_java_random_next_int(42, k) for k in range(4)] == [-1170105035, 234785527, -1360544799, 205897768]
    assert L.rts_java_random_next_int(0, 0) == -1155484576
    assert L.rts_java_random_next_double(42, 0) == 0.7275636800328681
    assert L.rts_java_random_next_int_bound(42, 10) == 0


@pytest.mark.parametrize("seed", [0, 1, 42, -7, 123456789, 2 ** 40 + 3])
def test_java_random_matches_restatement(seed):
    L = rtamd.scene_lib()
    r = PyJavaRandom(seed)
    ints = [r.next_int() for _ in range(16)]
    assert ints == [L.rts_java_random_next_int(seed, k) for k in range(16)]
    r = PyJavaRandom(seed)
    assert [r.next_double() for _ in range(8)] == [L.rts_java_random_next_double(seed, k) for k in range(8)]
    r = PyJavaRandom(seed)
    got = [L.rts_java_random_next_float(seed, k) for k in range(8)]
    assert [np.float32(r.next_float()) for _ in range(8)] == [np.float32(x) for x in got]


# --- scene builder ----------------------------------------------------------------------------

def _records(buf, size):
    assert len(buf) % size == 0
    return len(buf) // size


def _nodes(sc):
    raw = np.frombuffer(sc.buffers[S.BIND_BVH], dtype=np.uint8).reshape(-1, 32)
    box = raw[:, :24].copy().view(np.float32).reshape(-1, 6)
    ids = raw[:, 24:].copy().view(np.int32).reshape(-1, 2)
    return box, ids


@pytest.mark.parametrize("sid", list(range(10)))
def test_scene_layout(sid):
    sc = rtamd.Scene(sid, 64, 48, seed=1)
    info = sc.info
    for b, size in S.RECORD_BYTES.items():
        if b == S.BIND_LIGHTS:
            continue
        _records(sc.buffers[b], size)
    assert _records(sc.buffers[S.BIND_SPHERES], 48) == info["n_spheres"]
    assert _records(sc.buffers[S.BIND_QUADS], 80) == info["n_quads"]
    assert _records(sc.buffers[S.BIND_BOXES], 480) == info["n_boxes"]
    assert _records(sc.buffers[S.BIND_MEDIA], 20) == info["n_media"]
    assert _records(sc.buffers[S.BIND_BVH], 32) == info["n_bvh_nodes"]
    lights = sc.buffers[S.BIND_LIGHTS]
    n = struct.unpack_from("<i", lights, 0)[0]
    assert n == info["n_lights"] and len(lights) == 4 + 4 * n
    assert sc.camera.shape == (28,)
    assert info["max_stack"] <= 64 and info["bvh_depth"] <= 64


@pytest.mark.parametrize("sid", [0, 6, 7, 8])
def test_bvh_structure(sid):
    """Inner nodes (left type 0) contain their children's boxes; leaves hold prim pairs (BVHNode.java:24-45)."""
    sc = rtamd.Scene(sid, 64, 48, seed=1)
    box, ids = _nodes(sc)
    counts = {1: sc.info["n_spheres"], 2: sc.info["n_quads"], 3: sc.info["n_media"], 4: sc.info["n_boxes"]}
    seen = set()
    stack = [0]
    while stack:
        k = stack.pop()
        lt, rt = ids[k, 0] & 0xFFFF, ids[k, 1] & 0xFFFF
        li, ri = (ids[k, 0] >> 16) & 0xFFFF, (ids[k, 1] >> 16) & 0xFFFF
        if lt == 0:
            assert rt == 0, "inner node with a primitive right child"
            for c in (li, ri):
                assert np.all(box[c, 0::2] >= box[k, 0::2]) and np.all(box[c, 1::2] <= box[k, 1::2])
                stack += [c]
        else:
            assert li < counts[lt] and ri < counts[rt]
            seen.add((lt, li))
            seen.add((rt, ri))
    assert len(seen) == sc.info["n_bvh_prims"]


def test_scene8_inventory():
    """Book 2 final scene (Scene.java finalScene): 20x20 ground boxes, 1000-sphere cluster, 2 media."""
    sc = rtamd.Scene(8, 1920, 1080, seed=1)
    i = sc.info
    assert (i["n_boxes"], i["n_media"], i["n_spheres"], i["n_quads"]) == (400, 2, 1008, 1)
    assert i["n_bvh_nodes"] == 1793 and i["n_bvh_prims"] == 1409
    # finalScene never calls RaytraceModel.addLight (only cornellBox does, Scene.java:225,239):
    # the no-lights mixture-PDF case of SURVEY App. A Q1
    assert i["n_lights"] == 0
    assert any((t.width, t.height, t.format) == (1024, 512, S.TEX_RGB8) for t in sc.textures)   # earthmap
    assert any(t.format == S.TEX_R32F for t in sc.textures)                                      # perlin


def test_light_registration():
    """Only cornellBox registers lights: its ceiling quad and glass sphere (Scene.java:225,239)."""
    for sid in range(10):
        n = rtamd.Scene(sid, 16, 16, seed=1).info["n_lights"]
        assert n == (2 if sid == 6 else 0), (sid, n)
    lights = rtamd.Scene(6, 16, 16, seed=1).buffers[S.BIND_LIGHTS]
    packed = struct.unpack_from("<3i", lights, 0)
    assert packed[0] == 2 and {p >> 16 for p in packed[1:]} == {1, 2}   # type<<16|index: a sphere and a quad


def test_scene_is_seeded():
    a = rtamd.Scene(0, 32, 32, seed=5)
    b = rtamd.Scene(0, 32, 32, seed=5)
    c = rtamd.Scene(0, 32, 32, seed=6)
    assert a.buffers == b.buffers
    assert a.buffers[S.BIND_SPHERES] != c.buffers[S.BIND_SPHERES]


def test_camera_tracks_image_size():
    """Scene.updateCamera (Scene.java:37-41): the camera UBO follows the image aspect."""
    sc = rtamd.Scene(6, 600, 600, seed=1)
    cam0 = sc.camera.copy()
    sc.set_image_size(800, 400)
    assert sc.width == 800 and sc.height == 400
    assert abs(sc.camera[2] - 2.0) < 1e-6       # aspect_ratio
    assert not np.array_equal(cam0, sc.camera)


def test_bad_scene_id():
    with pytest.raises(ValueError):
        rtamd.Scene(42, 8, 8)


@pytest.mark.parametrize("spp", [1, 4, 10, 64, 4096])
def test_spp_uniforms(spp):
    """RaytraceExecutor.setSamplePerPixel: sqrtSpp = (float) Math.sqrt(spp); recip = 1f / sqrtSpp."""
    a, b = rtamd.spp_uniforms(spp)
    assert np.float32(a) == np.float32(math.sqrt(spp))
    assert np.float32(b) == np.float32(1.0) / np.float32(a)


# --- tonemap / PNG (Texture.saveAsPNG, Texture.java:89-120) ------------------------------------

def _tonemap_ref(rgba):
    c = rgba[..., :3].astype(np.float32)
    c = np.where(np.isnan(c), 0.0, c)
    u = np.where(c <= 0, 0, np.where(c >= 1, 255, np.rint(c * np.float32(255.0)))).astype(np.int64)
    lut = np.array([np.int8(np.int64(np.float32(np.float32(math.pow(b / 255.0, 1 / 2.2)) * np.float32(255.0)))
                            & 0xFF).view(np.uint8) for b in range(256)], np.uint8)
    return lut[u]


def test_tonemap_matches_restatement():
    rng = np.random.default_rng(3)
    img = rng.uniform(-0.2, 1.3, (17, 23, 4)).astype(np.float32)
    img[0, 0, 0] = np.nan
    img[1, 1, :] = np.inf
    assert np.array_equal(rtamd.tonemap_rgb8(img), _tonemap_ref(img))


def test_save_png_roundtrip(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(4)
    img = rng.uniform(0, 1, (9, 13, 4)).astype(np.float32)
    p = tmp_path / "out.png"
    rtamd.save_png(img, p)
    got = np.asarray(Image.open(p).convert("RGB"))
    assert np.array_equal(got, rtamd.tonemap_rgb8(img))
