"""HIP kernel vs CPU oracle, bit for bit (NaN positions equal), through the C ABI.

Every built-in scene of Scene.java (0-8) plus the build-defined scene 9, at sizes
the oracle finishes in seconds.  A fast kernel whose results differ from the
oracle's is not done.
"""
import numpy as np
import pytest

import rtamd
from helpers import bit_equal, gpu_image, mismatch_report, oracle_image

pytestmark = pytest.mark.gpu

CASES = [
    # scene, W, H, frames, depth
    (9, 40, 24, 8, 8),
    (6, 32, 32, 8, 5),
    (0, 48, 27, 6, 5),
    (8, 48, 27, 6, 5),
    (1, 32, 24, 4, 5),
    (2, 32, 24, 4, 5),
    (3, 32, 24, 4, 5),
    (4, 32, 24, 4, 5),
    (5, 32, 24, 4, 5),
    (7, 32, 32, 6, 5),
]


@pytest.mark.parametrize("scene_id,w,h,frames,depth", CASES)
def test_kernel_matches_oracle(gpu, scene_id, w, h, frames, depth):
    s = rtamd.Scene(scene_id, w, h, seed=1)
    ref = oracle_image(s, frames, max_depth=depth)
    out = gpu_image(s, frames, max_depth=depth)
    assert out.shape == ref.shape
    assert bit_equal(out, ref), mismatch_report(out, ref)


@pytest.mark.parametrize("scene_id", [3, 5, 8])
@pytest.mark.parametrize("packed", [1, 0])
def test_perlin_table_forms_match_oracle(gpu, scene_id, packed):
    """The Perlin noise (texture.glsl:38-94) from the packed LDS table (256 float4, perm entries
    as bytes: rt_kernel.hip perlin_noise_pk) and from the texture as uploaded (global memory),
    both bit for bit against the oracle; scenes 3, 5 and 8 carry Perlin textures."""
    s = rtamd.Scene(scene_id, 40, 30, seed=1)
    ref = oracle_image(s, 4, max_depth=5)
    out = gpu_image(s, 4, max_depth=5, options={"perlin_packed": packed})
    assert bit_equal(out, ref), mismatch_report(out, ref)


@pytest.mark.parametrize("scene_id,want", [(8, 1), (0, 0), (6, 0), (7, 0)])
def test_leaf_record_prefetch_matches_oracle(gpu, scene_id, want):
    """The compact-box kernels' leaf record prefetch (rt_kernel.hip leaf_prims_t, option
    leaf_prefetch): scene 8 (every box canonical; spheres, boxes and media staged in LDS) takes
    it, the others not (asserted); on and off, bit for bit against the oracle."""
    s = rtamd.Scene(scene_id, 48, 27, seed=1)
    ref = oracle_image(s, 6, max_depth=5)
    for opts, w in (({}, want), ({"leaf_prefetch": 0}, 0)):
        ctx = rtamd.RenderContext(options=opts)
        ctx.upload_scene(s)
        ctx.set_params(max_depth=5, spp=6)   # the oracle_image default: spp = frames
        ctx.resize(48, 27)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 6))
        out, info = ctx.read_image(), ctx.last_launch()
        ctx.close()
        assert info["leaf_prefetch"] == w, (opts, info)
        assert bit_equal(out, ref), f"{opts}: {mismatch_report(out, ref)}"


@pytest.mark.parametrize("shade", [1, 0])
@pytest.mark.parametrize("scene_id,w,h,frames,depth", CASES)
def test_shading_tables_match_oracle(gpu, scene_id, w, h, frames, depth, shade):
    """The shading tables in LDS (option shade_lds, default on: sphere records' third float4,
    compact boxes' materials with their face normals rebuilt from the compact record, texture
    descriptors and the small texture slots) and the records read from global memory (off):
    every scene bit for bit against the oracle; scene 8 stages all three tables (asserted)."""
    s = rtamd.Scene(scene_id, w, h, seed=1)
    ref = oracle_image(s, frames, max_depth=depth)
    ctx = rtamd.RenderContext(options={"shade_lds": shade})
    ctx.upload_scene(s)
    ctx.set_params(max_depth=depth, spp=frames)
    ctx.resize(w, h)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, frames))
    out, info = ctx.read_image(), ctx.last_launch()
    ctx.close()
    if scene_id == 8 or not shade:
        # scene 8 stages all three tables (beside the box pre-test nodes: the release kernels' 160 KB)
        assert info["shade_lds"] == 7 * shade, info
    assert bit_equal(out, ref), f"shade_lds {info['shade_lds']}: {mismatch_report(out, ref)}"


@pytest.mark.parametrize("scene_id,pairs", [(0, 1), (1, 1), (9, 1), (8, 0), (6, 0)])
def test_sphere_pair_kernel_matches_oracle(gpu, scene_id, pairs):
    """Scenes whose leaves are mostly two spheres take the kernels that test both at once
    (rt_kernel.hip leaf_prims_t SPAIR; scene 0's 485 spheres), the others not; with the option
    off every scene takes the plain kernels.  Both bit for bit against the oracle."""
    s = rtamd.Scene(scene_id, 48, 27, seed=1)
    ref = oracle_image(s, 4, max_depth=5)
    for opts, want in (({}, pairs), ({"sphere_pairs": 0}, 0)):
        ctx = rtamd.RenderContext(options=opts)
        ctx.upload_scene(s)
        ctx.set_params(max_depth=5, spp=4)
        ctx.resize(48, 27)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
        out, info = ctx.read_image(), ctx.last_launch()
        ctx.close()
        assert info["sphere_pairs"] == want, (opts, info)
        assert bit_equal(out, ref), f"{opts}: {mismatch_report(out, ref)}"


def test_chunked_frames_equal_single_launch(gpu):
    """n frames in one rt_render == the same frames over several rt_render calls."""
    s = rtamd.Scene(8, 40, 24, seed=3)
    a = gpu_image(s, 12, seed=5)
    b = gpu_image(s, 12, seed=5, chunks=[1, 4, 7])
    assert bit_equal(a, b), mismatch_report(a, b)


def test_multiframe_progressive_matches_oracle(gpu):
    """Running mean over frames 5..12 continuing a previous accumulation."""
    s = rtamd.Scene(6, 24, 24, seed=2)
    ref = oracle_image(s, 8, first_frame=5, spp=64)
    out = gpu_image(s, 8, first_frame=5, spp=64)
    assert bit_equal(out, ref), mismatch_report(out, ref)


SPECIALS = np.array([np.nan, 0.0, -0.0, np.inf, -np.inf, -1.0, -1e-30, 1e-45, 1e-40, 1.1754942e-38, 1.1754944e-38,
                     3.3732712e9, 3.3732714e9, -3.3732712e9, 1e10, -1e10, 3.4028235e38, -3.4028235e38,
                     2.5e7, 1.6777216e7, 1e-3, 0.7071067, 0.7071068, 1.0, 2.0], np.float32)


def test_builtins_bit_exact_on_device(gpu):
    """rt_glsl.h built-ins evaluated by gfx950 == evaluated by the x86 oracle."""
    import ctypes
    import pyoracle
    rng = np.random.default_rng(0)
    L = rtamd.amd()
    for name, lo, hi in [("sin", -3e5, 3e5), ("cos", -100, 100), ("log", 0, 1), ("acos", -1, 1), ("atan2", -5, 5),
                         ("fract", -1e4, 1e4), ("sqrt", 0, 1e6), ("inversesqrt", 0, 1e6)]:
        x = rng.uniform(lo, hi, 20000).astype(np.float32)
        # the branch-free special cases (rt_glsl.h g_log, g_sin / g_cos's parity of j): NaN,
        # signed zeros and infinities, negatives, subnormals, arguments past 2^24
        x[:SPECIALS.size] = SPECIALS
        y = rng.uniform(-5, 5, 20000).astype(np.float32)
        ref = pyoracle.eval_builtin(name, x, y)
        out = np.empty_like(x)
        fp = ctypes.POINTER(ctypes.c_float)
        rc = L.rt_debug_eval_builtin(0, pyoracle.BUILTINS[name], x.ctypes.data_as(fp), y.ctypes.data_as(fp),
                                     out.ctypes.data_as(fp), x.size)
        assert rc == 0
        assert bit_equal(out, ref), f"{name}: {mismatch_report(out[:, None], ref[:, None])}"


def test_shared_reciprocal_division_bit_exact(gpu):
    """rcp_nr / div_nr (rt_kernel.hip), the leaf tests' division by a shared
    reciprocal, give the bits of the compiler's '/' -- and of IEEE division
    (numpy) -- for every quotient in the regime the kernel uses them in: operands
    and quotient normal, numerator above 2^-103, exponents less than 96 apart.
    Also with the reciprocal of the negated denominator, negated (box faces)."""
    import ctypes
    rng = np.random.default_rng(7)
    L = rtamd.amd()
    n = 1 << 22
    num = (rng.choice([-1.0, 1.0], n) * np.exp2(rng.uniform(-100, 60, n)) * rng.uniform(1, 2, n)).astype(np.float32)
    den = (rng.choice([-1.0, 1.0], n) * np.exp2(rng.uniform(-62, 62, n)) * rng.uniform(1, 2, n)).astype(np.float32)
    # mantissas next to powers of two, where the reciprocal is least accurate
    k = n // 8
    den[:k] = (np.exp2(rng.integers(-30, 30, k)) * (1 + rng.integers(-64, 64, k) * 2.0 ** -23)).astype(np.float32)
    num[k:2 * k] = (np.exp2(rng.integers(-30, 30, k)) * (2 - rng.integers(1, 64, k) * 2.0 ** -23)).astype(np.float32)
    q64 = num.astype(np.float64) / den.astype(np.float64)
    en, ed = np.frexp(num)[1], np.frexp(den)[1]
    regime = ((np.abs(num) >= 2.0 ** -103) & (np.abs(den) >= 2.0 ** -125) & (np.abs(den) <= 2.0 ** 125) &
              (en - ed < 96) & (np.abs(q64) >= 2.0 ** -125) & (np.abs(q64) < 2.0 ** 127))
    assert regime.mean() > 0.8
    num, den = num[regime], den[regime]
    fp = ctypes.POINTER(ctypes.c_float)
    outs = {}
    for fn in (100, 101, 102):
        out = np.empty_like(num)
        assert L.rt_debug_eval_builtin(0, fn, num.ctypes.data_as(fp), den.ctypes.data_as(fp),
                                       out.ctypes.data_as(fp), num.size) == 0
        outs[fn] = out.view(np.uint32)
    ieee = (num / den).view(np.uint32)
    assert (outs[100] == ieee).all(), int((outs[100] != ieee).sum())
    for fn in (101, 102):
        bad = np.flatnonzero(outs[fn] != outs[100])
        assert bad.size == 0, (fn, bad.size, num[bad[:4]], den[bad[:4]])


@pytest.mark.parametrize("opts,expect", [({}, True), ({"box_vnodes": 0}, False), ({"box_pretest": 0}, False)])
def test_box_pretest_nodes_match_oracle(gpu, opts, expect):
    """Round 5: scene 8's ground boxes' bounds pre-tests run as nodes of the
    walk (option box_vnodes, on by default in the compact-box kernels when the pre-test is on);
    the leaf stage tests only the boxes they pass.  Bit for bit against the oracle either way, and
    the launch reports the chain nodes it walked."""
    s = rtamd.Scene(8, 48, 27, seed=1)
    ref = oracle_image(s, 6, max_depth=5)
    ctx = rtamd.RenderContext(devices=(0,), options=opts)
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=6)
    ctx.resize(48, 27)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 6))
    out = ctx.read_image()
    info = ctx.last_launch()
    ctx.close()
    assert (info["box_vnodes"] > 0) == expect, info
    if expect:   # one node per box of the all-box leaves (390 of scene 8's 400 boxes)
        from test_fast_tables import is_leaf, threaded
        n = sum((2 if (int(nd["meta"]) >> 20) & 0xF else 1) for nd in threaded(s)
                if is_leaf(nd) and (int(nd["meta"]) >> 16) & 0xF == 4 and (int(nd["meta"]) >> 20) & 0xF in (0, 4))
        assert info["box_vnodes"] == n == 390, (info, n)
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_collapsed_walk_matches_oracle_and_follows_the_camera(gpu):
    """Round 5: the link walk leaves out the inner nodes a grid of camera rays says cost more tests
    than they save (option collapse, on by default; rt_capi.hip plan_collapse).  Bit for bit against
    the oracle; the plan is the host's for this camera and image size, and a moved camera re-plans
    it (the launch reports the count the context-free planner gives for the new camera)."""
    from test_link_nodes import collapse_links
    s = rtamd.Scene(8, 48, 27, seed=1)
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=4)
    cams = [s.camera.copy(), s.camera.copy()]
    cams[1][4:7] += np.float32([40.0, 25.0, -30.0])   # the same view, translated
    cams[1][8:11] += np.float32([40.0, 25.0, -30.0])
    for cam in cams:
        s.override_camera(cam)
        ctx.set_camera(s.camera)
        ctx.resize(48, 27)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
        out = ctx.read_image()
        info = ctx.last_launch()
        _, _, nd = collapse_links(s, 48, 27, rebuild=2)
        assert info["collapsed"] == nd > 0, (info, nd)
        ref = oracle_image(s, 4, max_depth=5)
        assert bit_equal(out, ref), mismatch_report(out, ref)
    ctx.close()
