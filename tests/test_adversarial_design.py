"""The adversarial scenes (tests/adversarial.py) aim where they claim to, checked on the
CPU: the exact camera grids put ray hits on box edges and corners, at |d.y| around the
1e-8 cut and at t = tmin; the scaled scenes sit inside / past 2^20; the clouds' BVHs
pass 2047 nodes.  The oracle renders each (finite, not flat).  The GPU comparison is
tests/test_gpu_adversarial.py."""
import numpy as np
import pytest

import adversarial
import pyoracle
import rtamd

F32 = np.float32
CASES = {c.name: c for c in adversarial.cases()}


def camera_rays(scene):
    """Pixel rays of an exact grid camera (recip_sqrt_spp = 0), as the kernel computes them."""
    u = scene.camera
    o, ul, du, dv = u[4:7], u[8:11], u[12:15], u[16:19]
    W, H = scene.width, scene.height
    x = np.arange(W, dtype=F32)[None, :, None]
    y = np.arange(H, dtype=F32)[:, None, None]
    base = (ul + du * x) + dv * y
    coord = base + (du * F32(-0.5) + dv * F32(-0.5))
    return o, (coord - o).astype(F32)


def test_edges_grid_hits_edges_and_corners():
    o, d = camera_rays(CASES["edges"].scene)
    t = F32(4.0)                                  # box 1's front face z = -4
    p = o + d * t
    on_x = np.abs(np.abs(p[..., 0]) - 2) == 0    # x = +-2 edges
    on_y = np.abs(np.abs(p[..., 1]) - 1) == 0    # y = +-1 edges
    inside_y = np.abs(p[..., 1]) <= 1
    inside_x = np.abs(p[..., 0]) <= 2
    assert (on_x & inside_y).sum() >= 16 and (on_y & inside_x).sum() >= 16 and (on_x & on_y).sum() == 4


def test_grazing_rays_straddle_the_cut():
    _, d = camera_rays(CASES["grazing_grid"].scene)
    dy = np.abs(d[..., 1])
    assert (dy < F32(1e-8)).sum() > 0 and ((dy >= F32(1e-8)) & (dy < F32(2e-8))).sum() > 0
    _, d = camera_rays(CASES["grazing_cut"].scene)
    assert np.all(d[..., 1] == -F32(1e-8))
    _, d = camera_rays(CASES["grazing_below"].scene)
    assert np.all(np.abs(d[..., 1]) < F32(1e-8))


@pytest.mark.parametrize("name,rel", [("tmin_at", 0), ("tmin_below", -1), ("tmin_above", 1)])
def test_tmin_planes(name, rel):
    o, d = camera_rays(CASES[name].scene)
    t = (F32(0) - o[2]) / d[..., 2]                # the front face z = 0 (normal +z)
    tmin = F32(0.001)
    assert np.all(np.sign(t - tmin) == rel)


def test_extents_and_bvh_sizes():
    assert CASES["bvh_4k_lds"].scene.info["n_bvh_nodes"] > 2047
    assert CASES["bvh_9k_two_level"].scene.info["n_bvh_nodes"] * 32 > 152 * 1024
    for name, lo, hi in (("extent_inside_2^20", 0.9, 1.0), ("extent_past_2^20", 1.0, 1.2)):
        q = np.frombuffer(CASES[name].scene.buffers[4], np.float32).reshape(-1, 20)[:, 4:7]
        m = np.abs(q).max() / 2 ** 20
        assert lo < m < hi, (name, m)


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_renders_case(name):
    c = CASES[name]
    o = pyoracle.OracleScene(c.scene, max_depth=c.depth, uniforms=c.uniforms)
    img = pyoracle.render(o, rtamd.frame_rand_factors(1, 0, c.frames))
    assert np.isfinite(img).all() and img[..., :3].std() > 0
