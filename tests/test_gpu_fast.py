"""The exact near-first walk (A/B build variant 61, rt_kernel.hip trace_fast).

It must render the same bits as the reference-order walk: against the oracle
on every scene at small sizes, and against variant 0 (itself pinned to the
oracle, test_gpu_fullsize.py) on whole 1080p images of the scenes it runs on.
The diagnostic counters show that the walk is really taken and how often a
ray needs the exact walk instead.
"""
import ctypes

import pytest

import rtamd
from helpers import bit_equal, mismatch_report, oracle_image

pytestmark = pytest.mark.gpu

TRACES, EXACT, WHY, STEPS, TESTS = 21, 22, 23, 32, 33   # rt_kernel.hip ST_FAST_* (stats builds)


def render(variant, scene, frames, depth=5, spp=None, stats=False):
    ctx = rtamd.RenderContext(devices=(0,), options={"kernel_variant": variant}, ab=True)
    L = rtamd.amd_ab()
    if stats:
        assert L.rt_debug_enable_stats(ctx._h, 1) == 0
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=depth, spp=spp or frames)
    ctx.resize(scene.width, scene.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, frames))
    img = ctx.read_image()
    counters = None
    if stats:
        buf = (ctypes.c_ulonglong * 64)()
        assert L.rt_debug_read_stats(ctx._h, buf, 64) == 0
        counters = (buf[TRACES], buf[EXACT], [buf[WHY + r] for r in range(9)], buf[STEPS], buf[TESTS])
    ctx.close()
    return img, counters


@pytest.mark.parametrize("variant", [61])
@pytest.mark.parametrize("sid", range(10))
def test_fast_walk_matches_oracle(gpu, sid, variant):
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    out, _ = render(variant, scene, 4)
    ref = oracle_image(scene, 4)
    assert bit_equal(out, ref), mismatch_report(out, ref)


@pytest.mark.parametrize("variant", [61])
@pytest.mark.parametrize("sid,frames", [(8, 16), (0, 8), (2, 4), (3, 4), (5, 8), (9, 8)])
def test_fast_walk_equals_reference_walk_1080p(gpu, sid, frames, variant):
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    ref, _ = render(30, scene, frames)
    out, _ = render(variant, scene, frames)
    assert bit_equal(out, ref), mismatch_report(out, ref)


@pytest.mark.parametrize("variant", [61])
@pytest.mark.parametrize("sid,max_exact", [(8, 0.002), (0, 0.002)])
def test_fast_walk_is_taken(gpu, sid, max_exact, variant):
    scene = rtamd.Scene(sid, 640, 360, seed=1)
    _, (traces, exact, why, steps, tests) = render(variant, scene, 4, stats=True)
    print(f"variant {variant} scene {sid}: {traces} traces, {exact} took the exact walk ({exact / max(traces, 1):.5f}); "
          f"reasons 1-9 (1/dir inf, tie, leaf, tracker tie, tracker leaf, medium leaf, medium t, origin, stack): {why}; "
          f"{steps / max(traces, 1):.1f} node steps, {tests / max(traces, 1):.2f} prim tests per trace")
    assert traces > 640 * 360 * 4 and exact < max_exact * traces
