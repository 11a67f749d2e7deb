"""Adversarial parity: the kernel's exactness shortcuts against rays aimed at what
could break them (tests/adversarial.py), through the C ABI, bit for bit against
the CPU oracle.

The shortcuts and what each case aims at:
  * the box bounds pre-test (its margin argument): box edges and corners hit
    exactly, grazing faces, t at tmin, extents near 2^20;
  * the shared-reciprocal division (rcp_nr / div_nr): the same, with the regime
    check proven by a scene just inside 2^20 (on) and one just past (off);
  * the compact box records (box_test_compact): canonical boxes at exact edges,
    grazing and t = tmin; rotated boxes take the full records;
  * the link-format walk beyond 2047 nodes, in LDS (~4000 nodes) and two-level
    (~9800 nodes: top levels in LDS, the rest from global memory);
  * the spine entry (walks starting past the root's right spine): origins 0.0008 to
    0.01 inside the spine box's face and edge, where the entry's margin and the
    reference's own slab result change from pixel to pixel.
Every case renders with the default options and with each shortcut turned off
(rt_debug.h RT_OPTION_*); all must equal the oracle.  The launch each default
render took is asserted (rt_debug_last_launch), so a case cannot pass by
silently taking another path.
"""
import numpy as np
import pytest

import adversarial
import pyoracle
import rtamd
from helpers import bit_equal, mismatch_report

pytestmark = pytest.mark.gpu

CASES = adversarial.cases()
OFF = [{}, {"box_pretest": 0}, {"fastdiv": 0}, {"compact_boxes": 0}, {"spine": 0}, {"shade_lds": 0},
       {"box_vnodes": 0}, {"zero_dir_end": 0}, {"rebuild": 0}, {"collapse": 0, "rebuild": 0}]


def oracle(case):
    o = pyoracle.OracleScene(case.scene, max_depth=case.depth, uniforms=case.uniforms)
    return pyoracle.render(o, rtamd.frame_rand_factors(1, 0, case.frames))


def render(case, options=None):
    ctx = rtamd.RenderContext(devices=(0,), options=options)
    ctx.upload_scene(case.scene)
    ctx.set_params(max_depth=case.depth, uniforms=case.uniforms)
    ctx.resize(case.scene.width, case.scene.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, case.frames))
    img = ctx.read_image()
    info = ctx.last_launch()
    ctx.close()
    return img, info


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_adversarial_case_matches_oracle(gpu, case):
    ref = oracle(case)
    for opts in OFF:
        out, info = render(case, opts)
        assert bit_equal(out, ref), f"{case.name} {opts or 'default'}: {mismatch_report(out, ref)}"
        if not opts:
            for k, v in case.expect.items():
                assert info[k] == v, f"{case.name}: launch {k} = {info[k]}, expected {v} ({info})"
        elif "collapse" in opts and case.name.startswith("spine"):
            # the reference tree's chain (with collapse the chain's always-hit nodes are left out
            # of the walk instead): root + 5 right children (tests/adversarial.py spine_box)
            assert info["spine"] == 6, info
        elif "spine" in opts:
            assert info["spine"] == 0, info


@pytest.mark.parametrize("sid,spine", [(8, 11), (0, 0)])
def test_scenes_walks_skip_their_spine(gpu, sid, spine):
    """Scene 8's right spine (11 nodes, every box +-5000: the fog's boundary sphere sits in
    the right-most leaf) is skipped by the walks that start inside it; scene 0 has none
    (its camera sits on the root box's top face, and its surfaces lie outside the ground
    sphere's box).  The same bits as with the entry off and as the oracle."""
    s = rtamd.Scene(sid, 64, 48, seed=1)
    ref = pyoracle.render(pyoracle.OracleScene(s, max_depth=5, spp=4), rtamd.frame_rand_factors(1, 0, 4))
    # on the reference tree's links (with the inner-node rebuild and collapse, the defaults, the
    # chain is gone: the rebuilt tree splits the fog's leaf off at the root)
    for opts, want in (({"collapse": 0, "rebuild": 0}, spine), ({"collapse": 0, "rebuild": 0, "spine": 0}, 0)):
        ctx = rtamd.RenderContext(options=opts)
        ctx.upload_scene(s)
        ctx.set_params(max_depth=5, spp=4)
        ctx.resize(64, 48)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
        out, info = ctx.read_image(), ctx.last_launch()
        ctx.close()
        assert info["spine"] == want, info
        assert bit_equal(out, ref), f"{opts}: {mismatch_report(out, ref)}"


@pytest.mark.parametrize("tll,small", [(1, 1), (0, 1), (1, 0)])
@pytest.mark.parametrize("cap", [4096, 32768, 65536])
def test_two_level_walk_forced(gpu, cap, tll, small):
    """The ~4000-node cloud, which fits LDS, with only `cap` bytes of its nodes staged, its
    leaf records in LDS (tll 1) or global memory, and its 8 boxes' records in LDS (option
    tl_small_lds) or global memory: the same bits as the oracle whatever the split between
    LDS and global nodes."""
    case = next(c for c in CASES if c.name == "bvh_4k_lds")
    ref = oracle(case)
    out, info = render(case, {"lds_node_cap": cap, "tl_leaf_lds": tll, "tl_small_lds": small})
    assert info["shape_name"] == "link-two-level" and info["lds_nodes"] == cap // 32, info
    assert info["walk_frac"] == 32, info   # the two-level rounds (rt_capi.hip LDS plan)
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_watchdog_fault_is_reported(gpu):
    """A progress bound of 0 trips every wave's first check: rt_sync reports the fault
    (RT_ERR_DEVICE), and the context renders correctly again with the bound restored."""
    s = rtamd.Scene(8, 64, 48, seed=1)
    ref = pyoracle.render(pyoracle.OracleScene(s, max_depth=5, spp=4), rtamd.frame_rand_factors(1, 0, 4))
    ctx = rtamd.RenderContext(options={"watchdog_ms": 0})
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=4)
    ctx.resize(64, 48)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
    with pytest.raises(rtamd.RTError, match="watchdog") as e:
        ctx.sync()
    assert e.value.code == -2
    ctx.set_option("watchdog_ms", 120000)
    ctx.resize(64, 48)                     # a fresh zero image
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
    out = ctx.read_image()
    ctx.close()
    assert bit_equal(out, ref), mismatch_report(out, ref)


def test_chunk_wait_fault_is_reported(gpu):
    """Ordered one-frame chunks of one tile with a wait bound of 0: a wave that finds its
    tile's previous chunk unpublished stops waiting and sets the fault word."""
    s = rtamd.Scene(8, 8, 8, seed=1)
    ctx = rtamd.RenderContext(options={"chunk_wait_ms": 0, "stage_tiles": 0, "chunk_target": 100000})
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=256)
    ctx.resize(8, 8)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 256))
    with pytest.raises(rtamd.RTError, match="ordered-chunk wait") as e:
        ctx.sync()
    assert e.value.code == -2
    ctx.close()


def test_rand_factors_and_sizes_are_validated(gpu):
    """Inputs that would freeze rand() on the device (random.glsl:2-7) are rejected."""
    s = rtamd.Scene(6, 8, 8, seed=1)
    ctx = rtamd.RenderContext()
    ctx.upload_scene(s)
    ctx.set_params(max_depth=5, spp=4)
    ctx.resize(8, 8)
    for bad in (np.nan, np.inf, -np.inf, 2048.0):
        rf = rtamd.frame_rand_factors(1, 0, 3)
        rf[1] = bad
        with pytest.raises(rtamd.RTError, match="rand_factors"):
            ctx.render(1, rf)
    with pytest.raises(rtamd.RTError, match="bad image size"):
        ctx.resize(65537, 1)
    ctx.close()


def test_release_library_has_no_ab_options(gpu):
    """The release library: no kernel variants, no ablations, no stats kernels."""
    assert rtamd.amd().rt_debug_ab_build() == 0 and rtamd.amd_ab().rt_debug_ab_build() == 1
    ctx = rtamd.RenderContext()
    for name in ("kernel_variant", "debug_flags"):
        with pytest.raises(rtamd.RTError, match="unknown option"):
            ctx.set_option(name, 0)
    ctx.close()


@pytest.mark.parametrize("sid,want", [(6, 8), (0, 32), (8, 48)])
def test_walk_threshold_by_bvh_size(gpu, sid, want):
    """walk_frac 0 (the default) picks the walk round threshold by BVH size (rt_capi.hip
    walk_frac_for: 8/64 up to 64 nodes, 32 up to 1024, 48 above; measured per scene); explicit
    values override it.  Rounds only regroup lanes: the same bits at the default, 8 and 48."""
    scene = rtamd.Scene(sid, 96, 64, seed=1)
    imgs = []
    for v in (0, 8, 48):
        c = rtamd.RenderContext(options={"walk_frac": v})
        assert c.get_option("walk_frac") == v
        c.upload_scene(scene)
        c.set_params(max_depth=5, spp=4096)
        c.resize(96, 64)
        c.render(1, rtamd.frame_rand_factors(1, 0, 6))
        imgs.append(c.read_image())
        assert c.last_launch()["walk_frac"] == (v or want), c.last_launch()
        c.close()
    assert bit_equal(imgs[0], imgs[1]) and bit_equal(imgs[0], imgs[2]), f"scene {sid}"


def test_shading_threshold_by_kernel(gpu):
    """sm_frac 0 (the default) picks the threshold by kernel (50/64 for the compact-box kernels,
    56/64 else, rt_capi.hip); explicit values 1..64 override it and anything else is refused.
    The threshold only regroups which lanes shade together: scene 8 (compact boxes) and scene 6
    render the same bits at 0, 50 and 56."""
    ctx = rtamd.RenderContext()
    assert ctx.get_option("sm_frac") == 0
    for v in (-1, 65):
        with pytest.raises(rtamd.RTError, match="out of range"):
            ctx.set_option("sm_frac", v)
    ctx.close()
    for sid in (8, 6):
        scene = rtamd.Scene(sid, 160, 96, seed=1)
        imgs = []
        for v in (0, 50, 56):
            c = rtamd.RenderContext(options={"sm_frac": v})
            c.upload_scene(scene)
            c.set_params(max_depth=5, spp=4096)
            c.resize(160, 96)
            c.render(1, rtamd.frame_rand_factors(1, 0, 8))
            imgs.append(c.read_image())
            c.close()
        assert bit_equal(imgs[0], imgs[1]) and bit_equal(imgs[0], imgs[2]), f"scene {sid}"


@pytest.mark.parametrize("sid", [8, 0])
def test_non_nesting_bvh_under_default_options(gpu, sid):
    """an uploaded BVH whose inner boxes do not hold their children's (the ABI takes
    any BVH bytes).  Inner nodes are shrunk to a small box around their centre, so the
    reference's walk prunes their leaves for most rays; the inner-node rebuild and the collapse
    (both on by default) must then stand down -- a rebuilt tree would reach those leaves, and
    a medium's rand() draws would shift -- and the default render equals the oracle's walk of
    the uploaded tree bit for bit."""
    s = rtamd.Scene(sid, 64, 36, seed=1)
    rec = np.frombuffer(s.buffers[1], dtype=[("box", "<f4", 6), ("l", "<u4"), ("r", "<u4")]).copy()
    inner = [k for k in range(len(rec)) if rec[k]["l"] & 0xFFFF == 0 and rec[k]["r"] & 0xFFFF == 0]
    assert len(inner) > 60
    for k in inner[2:40:7]:
        b = rec[k]["box"].astype(np.float64)
        c, h = (b[0::2] + b[1::2]) / 2, (b[1::2] - b[0::2]) / 8
        rec[k]["box"] = np.stack([c - h, c + h], axis=1).reshape(6).astype(np.float32)
    s.buffers = dict(s.buffers)
    s.buffers[1] = rec.tobytes()
    case = type("Case", (), dict(scene=s, depth=5, uniforms=rtamd.spp_uniforms(4), frames=4))
    ref = oracle(case)
    out, info = render(case)
    assert bit_equal(out, ref), mismatch_report(out, ref)
    assert info["rebuilt"] == 0 and info["collapsed"] == 0, info
