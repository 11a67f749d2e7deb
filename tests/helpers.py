"""Shared helpers for the parity tests (test infrastructure)."""
import numpy as np

import pyoracle
import rtamd


def oracle_image(scene, frames, max_depth=5, spp=None, first_frame=1, seed=1, **kw):
    spp = spp or frames
    o = pyoracle.OracleScene(scene, max_depth=max_depth, spp=spp)
    rf = rtamd.frame_rand_factors(seed, first_frame - 1, frames)
    return pyoracle.render(o, rf, first_frame=first_frame, **kw)


def gpu_image(scene, frames, max_depth=5, spp=None, first_frame=1, seed=1, devices=(0,), chunks=None, options=None,
              ab=False):
    spp = spp or frames
    ctx = rtamd.RenderContext(devices=devices, options=options, ab=ab)
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=max_depth, spp=spp)
    ctx.resize(scene.width, scene.height)
    chunks = chunks or [frames]
    f = first_frame
    for n in chunks:
        ctx.render(f, rtamd.frame_rand_factors(seed, f - 1, n))
        f += n
    img = ctx.read_image()
    ctx.close()
    return img


def bit_equal(a, b):
    """Bitwise equality with every NaN treated as equal."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


def mismatch_report(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    diff = (a.view(np.uint32) != b.view(np.uint32)) & ~(np.isnan(a) & np.isnan(b))
    px = diff.any(axis=-1)
    n = int(px.sum())
    if n == 0:
        return "identical"
    ys, xs = np.nonzero(px)
    return f"{n} pixels differ (first at y={ys[0]} x={xs[0]}: {a[ys[0], xs[0]]} vs {b[ys[0], xs[0]]}); max|d|={np.nanmax(np.abs(a - b))}"
