"""Parity at BASELINE.json's full sizes (configs C2-C5), through the C ABI.

The oracle cannot render a whole 1080p/4K image in seconds, so each case renders
the full image on the GPU and checks it three ways:
  * sampled rows: the oracle renders a few whole 8-row stripes of the same image
    (its stripe partition: world = n_stripes, rank = stripe) and those rows must
    match the GPU image bit for bit;
  * work-split independence: one unit per tile (all frames of the launch in
    one wave) and tile x ordered frame-chunk units (the running mean handed
    from wave to wave through the image, rt_kernel.hip wait_chunk) give the
    same bits;
  * partition independence: N stripe-partitioned contexts (one per rank, as
    one process per GPU would run them) reassemble to the 1-context image.
"""
import numpy as np
import pytest

import pyoracle
import rtamd
from helpers import bit_equal, mismatch_report

pytestmark = pytest.mark.gpu

STRIPE = 8


def render(scene, frames, depth, spp, rank=0, world=1, stripe=16, options=None):
    ctx = rtamd.RenderContext(devices=(0,), rank=rank, world=world, stripe_rows=stripe, options=options)
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=depth, spp=spp)
    ctx.resize(scene.width, scene.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, frames))
    img = ctx.read_image()
    ctx.close()
    return img


def oracle_rows(scene, frames, depth, spp, stripes):
    """Oracle render of the given 8-row stripes only (rest of the image stays 0)."""
    o = pyoracle.OracleScene(scene, max_depth=depth, spp=spp)
    rf = rtamd.frame_rand_factors(1, 0, frames)
    n_stripes = (scene.height + STRIPE - 1) // STRIPE
    img = np.zeros((scene.height, scene.width, 4), np.float32)
    for s in stripes:
        pyoracle.render(o, rf, image=img, rank=s, world=n_stripes, stripe_rows=STRIPE)
    return img


def check_rows(gpu_img, ref, stripes, h):
    for s in stripes:
        r0, r1 = s * STRIPE, min(h, (s + 1) * STRIPE)
        assert bit_equal(gpu_img[r0:r1], ref[r0:r1]), f"rows {r0}-{r1}: {mismatch_report(gpu_img[r0:r1], ref[r0:r1])}"


# (config, scene, W, H, frames, spp uniform, depth)
CONFIGS = [
    ("C2 scene0 1080p", 0, 1920, 1080, 3, 1024, 5),
    ("C3 scene8 1080p", 8, 1920, 1080, 3, 4096, 5),
    ("C4 scene6 1080p", 6, 1920, 1080, 3, 4096, 5),
    ("C5 scene8 4K", 8, 3840, 2160, 2, 8192, 5),
]


@pytest.mark.parametrize("name,sid,w,h,frames,spp,depth", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_full_size_sampled_rows_match_oracle(gpu, name, sid, w, h, frames, spp, depth):
    scene = rtamd.Scene(sid, w, h, seed=1)
    n_stripes = (h + STRIPE - 1) // STRIPE
    rng = np.random.default_rng(sid * 7 + w)
    stripes = sorted({0, n_stripes - 1, *rng.choice(n_stripes, 3, replace=False).tolist()})
    direct = render(scene, frames, depth, spp, options={"chunk_target": 0})
    chunked = render(scene, frames, depth, spp, options={"chunk_target": 64})
    assert bit_equal(direct, chunked), "direct vs chunked: " + mismatch_report(direct, chunked)
    ref = oracle_rows(scene, frames, depth, spp, stripes)
    check_rows(direct, ref, stripes, h)
    assert np.isfinite(direct[..., 3]).all() and (direct[..., 3] == 1.0).all()


@pytest.mark.parametrize("world", [2, 8])
def test_full_size_stripe_partition_equals_one_gpu(gpu, world):
    """BASELINE C5's tile partition: the N-rank stripes reassemble to the 1-rank image."""
    scene = rtamd.Scene(8, 1920, 1080, seed=1)
    one = render(scene, 2, 5, 8192)
    parts = np.stack([
        np.pad(blk, ((0, rtamd.padded_local_rows(1080, world, STRIPE) - blk.shape[0]), (0, 0), (0, 0)))
        for blk in (render(scene, 2, 5, 8192, rank=r, world=world, stripe=STRIPE) for r in range(world))])
    full = rtamd.deinterleave(parts, 1080, world, STRIPE)
    assert bit_equal(full, one), mismatch_report(full, one)


@pytest.mark.parametrize("sid", [8, 0])
def test_ordered_chunks_equal_whole_launch_1080p(gpu, sid):
    """64 frames at 1080p as 64 one-frame chunks per tile (32 400 tiles, 63 wave-to-wave
    hand-offs each, every chunk on whichever CU/XCD dequeues it) == one unit per tile
    == 64 staged one-frame chunks per tile (the default's split, at its extreme)."""
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    whole = render(scene, 64, 5, 4096, options={"chunk_target": 0})
    chunked = render(scene, 64, 5, 4096, options={"stage_tiles": 0, "chunk_target": 100000})
    assert bit_equal(chunked, whole), mismatch_report(chunked, whole)
    staged = render(scene, 64, 5, 4096, options={"staged_chunk_target": 100000, "chunk_target": 16})
    assert bit_equal(staged, whole), mismatch_report(staged, whole)


@pytest.mark.parametrize("sid", [8, 6, 7])
@pytest.mark.parametrize("knob", ["box_pretest", "fastdiv", "compact_boxes"])
def test_exactness_shortcuts_change_no_bit_1080p(gpu, knob, sid):
    """The box bounds pre-test, the shared-reciprocal divisions and the compact box records
     against the plain tests, whole 1080p images (every ray of 8 frames): scene 8
    (ground boxes seen at grazing angles), 6 and 7 (rotated boxes): the same bits."""
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    on = render(scene, 8, 5, 4096)
    off = render(scene, 8, 5, 4096, options={knob: 0})
    assert bit_equal(on, off), mismatch_report(on, off)


@pytest.mark.parametrize("world,rank", [(1, 0), (8, 3)])
@pytest.mark.parametrize("sid", [8, 0, 6])
def test_sparse_staging_changes_no_bit_1080p(gpu, sid, world, rank):
    """Sparse staging: every sample writes a flag byte and only the colours that are
    not exactly zero their 16 bytes; fold_kernel reads a clear flag back as the zero colour.
    Against dense staging, whole 1080p images of 16 frames continuing an
    accumulation (and one rank of 8 over 96 frames), the same bits; the default launch must
    have taken the sparse form."""
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    imgs = []
    for opts in ({}, {"sparse_stage": 0}):
        ctx = rtamd.RenderContext(devices=(0,), rank=rank, world=world, stripe_rows=8, options=opts)
        ctx.upload_scene(scene)
        ctx.set_params(max_depth=5, spp=4096)
        ctx.resize(1920, 1080)
        ctx.render(1, rtamd.frame_rand_factors(1, 0, 4))
        ctx.render(5, rtamd.frame_rand_factors(1, 4, 16 if world == 1 else 96))
        info = ctx.last_launch()
        imgs.append(ctx.read_image())
        ctx.close()
        assert info["staged"] == 1 and info["sparse"] == (0 if opts else 1), info
    assert bit_equal(imgs[0], imgs[1]), mismatch_report(imgs[0], imgs[1])


@pytest.mark.parametrize("sid", [8, 0])
@pytest.mark.parametrize("knob", ["big_wg", "sph_lds"])
def test_lds_record_copies_change_no_bit_1080p(gpu, knob, sid):
    """The leaf tests' records read from LDS: scene 8 runs as one 1024-thread
    workgroup per CU with its spheres' and canonical boxes' records staged beside the nodes,
    scene 0 stages its spheres in the 512-thread shape.  Against the global-memory reads
    (knob = 0), whole 1080p images of 8 frames: the same bits."""
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    on = render(scene, 8, 5, 4096)
    off = render(scene, 8, 5, 4096, options={knob: 0})
    assert bit_equal(on, off), mismatch_report(on, off)


# Walk structure / scheduling options against the default, whole 1080p images of 8 frames
# (the small-image suite once passed a walk that diverged at full size, so
# every non-default walk or scheduling form is gated here, bit for bit).
WALK_OPTIONS = [
    ("sm_frac", {"sm_frac": 8}), ("sm_frac", {"sm_frac": 64}), ("sm_batch", {"sm_batch": 16}),
    ("walk_frac", {"walk_frac": 16}), ("walk_frac", {"walk_frac": 48}), ("walk_frac", {"walk_frac": 64}),
    ("sphere_pairs", {"sphere_pairs": 0}), ("spine", {"spine": 0}), ("leaf_prefetch", {"leaf_prefetch": 0}),
    ("shade_lds", {"shade_lds": 0}), ("box_vnodes", {"box_vnodes": 0}), ("zero_dir_end", {"zero_dir_end": 0}),
    ("collapse", {"collapse": 0}), ("rebuild", {"rebuild": 0}), ("rebuild", {"rebuild": 0, "collapse": 0}),
    ("two_level", {"lds_node_cap": 16384}), ("two_level_leaf_global", {"lds_node_cap": 16384, "tl_leaf_lds": 0}),
    ("tail_chunks", {"tail_chunks": 0}), ("tail_chunks", {"tail_chunks": 7}),
]


@pytest.mark.parametrize("sid", [8, 0, 6])
@pytest.mark.parametrize("name,opts", WALK_OPTIONS, ids=[f"{n}-{list(o.values())[-1]}" for n, o in WALK_OPTIONS])
def test_walk_and_schedule_options_change_no_bit_1080p(gpu, sid, name, opts):
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    base = render(scene, 8, 5, 4096)
    other = render(scene, 8, 5, 4096, options=opts)
    assert bit_equal(base, other), f"{name} {opts}: " + mismatch_report(base, other)
