"""The link-format node loop (RT_KERNEL_VARIANT=37, rt_kernel.hip trace with
WHILE_WHILE bit 8; nodes from rt_capi.hip build_links).

It walks the reference's threaded BVH in the same node order as variant 30,
only with explicit hit / miss successors and packed slab arithmetic, so the
images must be identical bit for bit: against the oracle on every scene
(test_gpu_boundary.py VARIANTS) and against variant 30 on whole 1080p images
here.
"""
import pytest

import rtamd
from helpers import bit_equal, mismatch_report

pytestmark = pytest.mark.gpu


def render(monkeypatch, variant, scene, frames, depth=5):
    monkeypatch.setenv("RT_KERNEL_VARIANT", str(variant))
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=depth, spp=frames)
    ctx.resize(scene.width, scene.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, frames))
    img = ctx.read_image()
    ctx.close()
    return img


@pytest.mark.parametrize("sid,frames", [(8, 16), (0, 8), (2, 4), (6, 4), (9, 8)])
def test_link_walk_equals_threaded_walk_1080p(gpu, monkeypatch, sid, frames):
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    ref = render(monkeypatch, 30, scene, frames)
    out = render(monkeypatch, 37, scene, frames)
    assert bit_equal(out, ref), mismatch_report(out, ref)
