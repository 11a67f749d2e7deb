"""Parity anchors against the reference's own published renders (galleries/*.png).

The reference cannot run here; its only outputs are the gallery
PNGs, summarised in tests/golden/gallery.json by tests/golden/make_gallery_fixture.py
(the reference files are read there, once, never by these tests).  These tests
render with the CPU oracle, which the -m gpu suite pins bit for bit to the HIP
kernel, through the reference's PNG pipeline (rtamd.tonemap_rgb8 / save_png =
Texture.saveAsPNG, Texture.java:89-120).

Scene 0 (Book-1 final, Scene.java:43-105), exact bytes:
  * every open-sky pixel is the background (0.7, 0.8, 1.0) (Scene.java:104)
    through the running mean and saveAsPNG: the gallery's (217, 230, 255);
  * the sky/not-sky split of rows 0-135 (camera framing, the three fixed big
    spheres, the horizon) matches the gallery's pixel for pixel except at edges.
Scene 8 (Book-2 final, Scene.java:282-343), statistics over the regions whose
geometry is fixed (tests/gallery_regions.py; the ground boxes, the 1000-sphere
cluster and the moving sphere are masked out):
  * light quad: saturated (255, 255, 255) in both;
  * glass, metal, blue fog, earth and Perlin spheres: the mean of the
    linearised bytes, (b/255)^2.2, within LIN_TOL (relative, per channel) of the
    gallery's -- fog density (with SURVEY App. A Q7), dielectric, fuzzy metal,
    image and Perlin textures and the no-light Q1 decision all set these;
  * earth: the texture's pattern (8x8-pixel block means with a quadratic
    lighting trend removed) correlates >= EARTH_MIN_CORR with the gallery's per
    channel -- get_sphere_uv and the image texture's orientation and filtering
    (texture.glsl:96-132).  A left-right mirrored earth scores ~0.1-0.2.
Stated tolerance: per channel, region means of the linearised
bytes within 20 %; the measured worst case is 12 % (glass, green) at 256 spp.
"""
import base64
import json
import os

import numpy as np
import pytest

import gallery_regions as gr
import pyoracle
import rtamd

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "gallery.json")))

LIN_TOL = 0.20
EARTH_MIN_CORR = 0.80


def _render_rows(scene, spp, rows, stripe=8, depth=5):
    """Oracle render of the 8-row stripes covering `rows` (the rest stays 0)."""
    o = pyoracle.OracleScene(scene, max_depth=depth, spp=spp)
    rf = rtamd.frame_rand_factors(1, 0, spp)
    img = np.zeros((scene.height, scene.width, 4), np.float32)
    n_stripes = (scene.height + stripe - 1) // stripe
    for s in sorted({r // stripe for r in rows}):
        pyoracle.render(o, rf, image=img, rank=s, world=n_stripes, stripe_rows=stripe)
    return img


@pytest.fixture(scope="module")
def scene0_top():
    fx = FIX["scene0_sky"]
    sc = rtamd.Scene(0, fx["width"], 600, seed=1)
    img = _render_rows(sc, 64, range(fx["rows"]))
    return sc, img[:fx["rows"]]


def test_scene0_sky_is_the_gallery_colour(scene0_top, tmp_path):
    """Rows 0-38 are open sky in the gallery: all (217, 230, 255).  Ours, through
    the PNG writer, byte for byte."""
    fx = FIX["scene0_sky"]
    _, img = scene0_top
    full = fx["full_rows"]
    png = tmp_path / "sky.png"
    rtamd.save_png(img[:full], str(png))
    from test_cli import read_png
    got = read_png(str(png))
    assert got.shape == (full, fx["width"], 3)
    assert (got == np.array(fx["rgb"], np.uint8)).all(), np.unique(got.reshape(-1, 3), axis=0)[:5]
    # the sky is the background itself: every sample of these pixels missed every object
    assert np.allclose(img[:full, :, :3], [0.7, 0.8, 1.0], rtol=1e-5, atol=0)


def test_scene0_sky_mask_matches_gallery(scene0_top):
    """Rows 0-135: which pixels are exactly the sky colour -- the camera (Camera.java,
    Scene.java:98-102: vfov 20 from (13,2,3) to (0,0,0)), the three big spheres (Scene.java:85-92) and
    the horizon -- agrees with the gallery except along silhouettes (defocus blur,
    jitter) and the gallery's own random small spheres near the horizon."""
    fx = FIX["scene0_sky"]
    _, img = scene0_top
    rows, w = fx["rows"], fx["width"]
    gal = np.unpackbits(np.frombuffer(base64.b64decode(fx["mask_packbits_b64"]), np.uint8))[:rows * w]
    gal = gal.reshape(rows, w).astype(bool)
    ours = np.all(rtamd.tonemap_rgb8(img) == np.array(fx["rgb"], np.uint8), axis=-1)
    agree = float((ours == gal).mean())
    assert agree >= 0.97, f"sky mask agreement {agree:.4f}"
    assert ours.sum() > 0.5 * gal.sum()


@pytest.fixture(scope="module")
def scene8_small():
    """Scene 8 at a quarter of the gallery's size (200x150), 256 spp: region means."""
    sc = rtamd.Scene(8, 200, 150, seed=1)
    o = pyoracle.OracleScene(sc, max_depth=5, spp=256)
    img = pyoracle.render(o, rtamd.frame_rand_factors(1, 0, 256))
    return sc, img


def test_scene8_regions_match_gallery(scene8_small):
    sc, img = scene8_small
    fx = FIX["scene8_regions"]["regions"]
    regs = gr.scene8_regions(sc.camera, sc.width, sc.height, erode=1)
    lin = np.clip(np.nan_to_num(img[..., :3], nan=0.0), 0.0, 1.0)   # what the PNG bytes linearise to
    t8 = rtamd.tonemap_rgb8(img)
    assert fx["light"]["all_255"] and (t8[regs["light"]] == 255).all()
    report = {}
    for name in ("glass", "metal", "blue_fog", "earth", "perlin"):
        m = regs[name]
        assert m.sum() > 300, name
        ours = lin[m].mean(0)
        ratio = ours / np.array(fx[name]["lin_mean"])
        report[name] = np.round(ratio, 3).tolist()
    bad = {k: v for k, v in report.items() if max(abs(x - 1.0) for x in v) > LIN_TOL}
    assert not bad, f"region mean ratio outside 1 +- {LIN_TOL}: {bad} (all: {report})"


def test_scene8_earth_texture_pattern_matches_gallery():
    """The earth sphere's continents: 8x8 block means of the linearised image with a
    quadratic lighting trend removed, per channel, against the gallery's."""
    fx = FIX["scene8_earth_blocks"]
    B = fx["block"]
    sc = rtamd.Scene(8, 800, 600, seed=1)
    regs = gr.scene8_regions(sc.camera, 800, 600)
    blocks = gr.block_grid(regs["earth"], B)
    assert [list(b) for b in blocks] == fx["coords"]   # same masks as the fixture's
    rows = range(min(y for y, _ in blocks), max(y for y, _ in blocks) + B)
    img = _render_rows(sc, 64, rows)
    ours = gr.block_means(np.clip(img[..., :3], 0.0, 1.0), blocks, B)
    gal = np.array(fx["lin_means"])
    yx = np.array(blocks, float) + B / 2
    X = np.stack([np.ones(len(yx)), yx[:, 0], yx[:, 1], yx[:, 0] ** 2, yx[:, 1] ** 2, yx[:, 0] * yx[:, 1]], 1)

    def resid(v):
        coef, *_ = np.linalg.lstsq(X, v, rcond=None)
        return v - X @ coef
    corr = [float(np.corrcoef(resid(ours[:, c]), resid(gal[:, c]))[0, 1]) for c in range(3)]
    assert min(corr) >= EARTH_MIN_CORR, corr


@pytest.mark.gpu
def test_scene0_sky_through_the_kernel(gpu, scene0_top):
    """The same sky rows rendered by the HIP kernel through rt.h: the bits of the oracle's
    rows, hence the gallery's sky bytes."""
    sc, ref = scene0_top
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.upload_scene(sc)
    ctx.set_params(max_depth=5, spp=64)
    ctx.resize(sc.width, sc.height)
    ctx.render(1, rtamd.frame_rand_factors(1, 0, 64))
    out = ctx.read_image()[:ref.shape[0]]
    ctx.close()
    from helpers import bit_equal, mismatch_report
    assert bit_equal(out, ref), mismatch_report(out, ref)
    full = FIX["scene0_sky"]["full_rows"]
    assert (rtamd.tonemap_rgb8(out[:full]) == np.array(FIX["scene0_sky"]["rgb"], np.uint8)).all()


# Per-region tolerance of the 800x600 / 4096 spp / depth 6 comparison, from data
# (profiles/r03_gallery_seed_probe_png.log: seeds 1-8 through the PNG pipeline): the
# 8-seed mean distance from the gallery plus 3 seed-to-seed standard deviations, rounded
# up.  Glass refracts the unseeded cluster (sd 6-7%); earth (+4.1..5.6%) and metal
# (-4.4..6.0%) keep a systematic distance that neither the seed (sd <= 1.5%), the sample
# count (means move < 1% from 512 to 4096 spp; the gallery's pixel noise says ~6-8k spp,
# profiles/r03_gallery_spp_probe.log), the depth, nor light sampling (registering the
# light quad moves earth to 1.52, profiles/r03_gallery_light_probe.log) accounts for
# (DESIGN.md §2).
# Round 6: the metal offset is attributed -- the book's earlier metal scatter,
# reflect(unit(dir)) + fuzz * random_in_unit_sphere, instead of the reference sources' normalised
# reflection + fuzz * random_unit_vector (scatter.glsl:12-15), moves the metal region by x1.049-1.051
# and nothing else (tools/scene8_residual_probe.py --r6, profiles/r06_scene8_residual_probe.log:
# 0.942 -> 0.988 of the gallery): the gallery was rendered with that form.  So the product's metal
# region is expected at 1 / 1.049 = 0.953 of the gallery, within the seed data's spread about it
# (0.940-0.956, sd 0.015) + 3 sd: 6% (was 11% about 1.0).  Earth stays unattributed.
GPU_REGION_CENTRE = {"glass": 1.0, "metal": 0.953, "blue_fog": 1.0, "earth": 1.0, "perlin": 1.0}
GPU_REGION_TOL = {"glass": 0.24, "metal": 0.06, "blue_fog": 0.04, "earth": 0.07, "perlin": 0.04}
LIN_RAW_TOL = 0.08   # every region, raw floats in the linear domain (round 2's single bound)


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["reference", "sah"])
def test_scene8_regions_match_gallery_full_size_gpu(gpu, bvh):
    """Scene 8 at the gallery's own size (800x600) and 4096 spp through the HIP kernel
    (bit-exact with the oracle by the rest of the -m gpu suite): the fixed-geometry regions'
    means of the linearised bytes against book2_final(scene8).png, our image taken through
    the same PNG pipeline (rtamd.tonemap_rgb8 = Texture.saveAsPNG) and linearised the same
    way, and the earth texture's pattern.  The reference records neither the gallery's spp
    nor its max_depth (GUI slider 1-50, CLI default 5).  The blue fog region's blue channel
    pins the depth: 0.881 of the gallery at depth 5, 1.003 at 6, 1.105 at 7
    (tools/gallery_depth_probe.py, profiles/r02_gallery_depth_probe.log).  Tolerances:
    GPU_REGION_TOL.  Also in the non-parity fast mode (bvh "sah", rt_set_bvh_mode): the same
    anchors hold for the SAH tree's image (row f3's statistical gate)."""
    sc = rtamd.Scene(8, 800, 600, seed=1)
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.set_bvh_mode(bvh)
    ctx.upload_scene(sc)
    ctx.set_params(max_depth=6, spp=4096)
    ctx.resize(800, 600)
    rf = rtamd.frame_rand_factors(1, 0, 4096)
    for k in range(0, 4096, 512):
        ctx.render(k + 1, rf[k:k + 512])
    img = ctx.read_image()
    assert ctx.last_launch()["bvh_mode"] == rtamd.render.BVH_MODES[bvh]
    ctx.close()
    fx = FIX["scene8_regions"]["regions"]
    regs = gr.scene8_regions(sc.camera, 800, 600)
    t8 = rtamd.tonemap_rgb8(img)
    lin_png = (t8.astype(np.float64) / 255.0) ** 2.2
    assert (t8[regs["light"]] == 255).all()
    report = {}
    for name in ("glass", "metal", "blue_fog", "earth", "perlin"):
        ratio = lin_png[regs[name]].mean(0) / np.array(fx[name]["lin_mean"])
        report[name] = np.round(ratio, 3).tolist()
    print(f"scene 8 ({bvh} BVH), 800x600, 4096 spp, depth 6, region mean / gallery (PNG pipeline):", report)
    bad = {k: v for k, v in report.items() if max(abs(x - GPU_REGION_CENTRE[k]) for x in v) > GPU_REGION_TOL[k]}
    assert not bad, f"region mean ratio outside GPU_REGION_CENTRE +- GPU_REGION_TOL: {bad} (all: {report})"
    # The linear-domain bound kept beside the per-region PNG tolerances: the raw
    # floats, clipped to [0, 1], of every region -- glass included -- within 8% of the gallery's
    # linearised means.  This render is seed 1's, bit-exact by the rest of the suite; measured
    # worst 6.4% (earth; glass 4.6-5.5%, profiles/r03_gallery_seed_probe_raw.log seed 1, depth 6),
    # so a dielectric / refraction regression the glass region's 24% PNG-pipeline band (which
    # covers the unseeded cluster's seed-to-seed spread) would let through still fails here.
    lin_raw = np.clip(np.nan_to_num(img[..., :3].astype(np.float64), nan=0.0), 0.0, 1.0)
    raw = {name: np.round(lin_raw[regs[name]].mean(0) / np.array(fx[name]["lin_mean"]), 4).tolist()
           for name in ("glass", "metal", "blue_fog", "earth", "perlin")}
    print("raw linear region mean / gallery:", raw)
    bad_raw = {k: v for k, v in raw.items() if max(abs(x - 1.0) for x in v) > LIN_RAW_TOL}
    assert not bad_raw, f"raw linear region mean ratio outside {LIN_RAW_TOL}: {bad_raw}"
    lin = np.clip(np.nan_to_num(img[..., :3], nan=0.0), 0.0, 1.0)
    fe = FIX["scene8_earth_blocks"]
    B = fe["block"]
    blocks = [tuple(b) for b in fe["coords"]]   # the fixture's blocks (test above: the same masks)
    ours = gr.block_means(lin, blocks, B)
    gal = np.array(fe["lin_means"])
    yx = np.array(blocks, float) + B / 2
    X = np.stack([np.ones(len(yx)), yx[:, 0], yx[:, 1], yx[:, 0] ** 2, yx[:, 1] ** 2, yx[:, 0] * yx[:, 1]], 1)

    def resid(v):
        coef, *_ = np.linalg.lstsq(X, v, rcond=None)
        return v - X @ coef
    corr = [float(np.corrcoef(resid(ours[:, c]), resid(gal[:, c]))[0, 1]) for c in range(3)]
    print("earth pattern correlation per channel:", np.round(corr, 3).tolist())
    assert min(corr) >= 0.95, corr   # measured 0.985-0.991 (EARTH_MIN_CORR is for 64 spp)


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["reference", "sah"])
def test_scene6_blocks_match_gallery_4096spp_gpu(gpu, bvh):
    """The Cornell box (book3_final(scene6).png, 600x600, the CLI's depth 5) at 4096 spp
    through the HIP kernel: 60x60 block means of the PNG bytes against the gallery's, the
    per-channel statement of the CPU suite's 64 spp oracle check (tests/test_oracle.py::
    test_gallery_scene6) with the sampling noise gone."""
    B = FIX["block"]
    gb = np.array(FIX["scene6_block_means"])
    sc = rtamd.Scene(6, FIX["width"], FIX["height"], seed=1)
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.set_bvh_mode(bvh)
    ctx.upload_scene(sc)
    ctx.set_params(max_depth=5, spp=4096)
    ctx.resize(FIX["width"], FIX["height"])
    rf = rtamd.frame_rand_factors(1, 0, 4096)
    for k in range(0, 4096, 512):
        ctx.render(k + 1, rf[k:k + 512])
    img = ctx.read_image()
    ctx.close()
    ours = rtamd.tonemap_rgb8(img).astype(np.float64)
    h, w = ours.shape[:2]
    ob = ours.reshape(h // B, B, w // B, B, 3).mean(axis=(1, 3))
    d = ob - gb
    corr = float(np.corrcoef(gb.ravel(), ob.ravel())[0, 1])
    per_ch = [float(np.abs(d[..., c]).mean()) for c in range(3)]
    print(f"scene 6 ({bvh} BVH), 600x600, 4096 spp: corr", round(corr, 5), "mean |block diff| per channel (of 255)",
          np.round(per_ch, 3).tolist(), "max", round(float(np.abs(d).max()), 3))
    # measured: corr 0.99998, mean |diff| 0.133 / 0.139 / 0.136 of 255, max 0.79
    assert corr > 0.9999, corr
    assert max(per_ch) < 0.5, per_ch
    assert np.abs(d).max() < 2.0, np.abs(d).max()


def _render_gpu(sid, w, h, spp, depth, bvh="reference"):
    sc = rtamd.Scene(sid, w, h, seed=1)
    ctx = rtamd.RenderContext(devices=(0,))
    ctx.set_bvh_mode(bvh)
    ctx.upload_scene(sc)
    ctx.set_params(max_depth=depth, spp=spp)
    ctx.resize(w, h)
    rf = rtamd.frame_rand_factors(1, 0, spp)
    for k in range(0, spp, 512):
        ctx.render(k + 1, rf[k:k + 512])
    img = ctx.read_image()
    ctx.close()
    return sc, img


@pytest.mark.gpu
@pytest.mark.parametrize("bvh", ["reference", "sah"])
def test_scene0_fixed_spheres_match_gallery_gpu(gpu, bvh):
    """Scene 0's three fixed spheres (book1_final(scene0).png, 800x600) at 4096 spp through
    the HIP kernel: means of the linearised bytes over the pixels whose ray meets them above
    the random small spheres' layer, at the CLI's depth 5 (depth 6 moves glass from 1.09-1.12
    to 1.13-1.16 of the gallery).  The diffuse sphere is lit by the sky and the ground
    through the no-light mixture PDF, so its brightness checks that
    decision: measured 1.010-1.016 of the gallery; the metal sphere 1.003-1.007.  The glass
    sphere refracts the unseeded small spheres (not the gallery's): 1.09-1.12."""
    depth = 5
    fx = FIX["scene0_regions"]
    sc, img = _render_gpu(0, fx["width"], fx["height"], 4096, depth, bvh)
    regs = gr.scene0_regions(sc.camera, fx["width"], fx["height"])
    lin = np.clip(np.nan_to_num(img[..., :3], nan=0.0), 0.0, 1.0)
    report = {}
    for name, r in fx["regions"].items():
        m = regs[name]
        assert abs(int(m.sum()) - r["n_pixels"]) == 0, name   # the fixture's masks
        report[name] = np.round(lin[m].mean(0) / np.array(r["lin_mean"]), 3).tolist()
    print(f"scene 0 ({bvh} BVH), 800x600, 4096 spp, depth {depth}, region mean / gallery:", report)
    assert max(abs(x - 1.0) for n in ("diffuse", "metal") for x in report[n]) <= 0.03, report
    assert max(abs(x - 1.0) for x in report["glass"]) <= LIN_TOL, report
