"""The link-format node loop of the A/B build's variant 37 (rt_kernel.hip trace;
nodes from rt_capi.hip build_links) against the threaded meta-word walk (30).

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


def render(variant, scene, frames, depth=5):
    ctx = rtamd.RenderContext(devices=(0,), options={"kernel_variant": variant}, ab=True)
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=depth, spp=frames)
    ctx.resize(scene.width, scene.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, frames))
    img = ctx.read_image()
    ctx.close()
    return img


@pytest.mark.parametrize("sid,frames", [(8, 16), (0, 8), (2, 4), (6, 4), (9, 8)])
def test_link_walk_equals_threaded_walk_1080p(gpu, sid, frames):
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    ref = render(30, scene, frames)
    out = render(37, scene, frames)
    assert bit_equal(out, ref), mismatch_report(out, ref)
