"""Pixel masks of the reference galleries' deterministic regions (TEST INFRASTRUCTURE).

The reference's gallery renders (galleries/*.png, 800x600) used unseeded scene
geometry for scenes 0 and 8 (Math.random), so only the
objects whose geometry is fixed in Scene.java can be compared pixel-region by
pixel-region with this build's renders.  This module computes, per pixel, which
of those objects the pixel-centre camera ray meets first, from the scene's own
camera record (Camera.java:91-143 as packed in the UBO, rtamd.Scene.camera) and
the object list of Scene.java:282-343 (scene 8), excluding every pixel whose
ray may first meet unseeded geometry (the ground boxes, up to y = 101, and the
1000-sphere cluster) or the motion-blurred sphere.  Used by
tests/golden/make_gallery_fixture.py (which reads the galleries once, in this
container) and by tests/test_gallery_anchor.py (which reads only the committed
fixture).  Pure numpy; no reference files are read here.
"""
import numpy as np

# Scene.java:300-327 (scene 8): the deterministic spheres (centre, radius); the
# ConstantMedium boundaries are the spheres that carry them
SCENE8_SPHERES = {
    "glass": ((260.0, 150.0, 45.0), 50.0),        # Dielectric(1.5)
    "metal": ((0.0, 150.0, 145.0), 50.0),         # Metal(0.8, 0.8, 0.9; fuzz 0.999)
    "blue_fog": ((360.0, 150.0, 145.0), 70.0),    # Dielectric boundary + ConstantMedium(0.2)
    "earth": ((400.0, 200.0, 400.0), 100.0),      # ImageTexture earthmap
    "perlin": ((220.0, 280.0, 300.0), 80.0),      # PerlinNoiseTexture(0.2)
}
# light quad Q=(123,554,147), u=(300,0,0), v=(0,0,265) (Scene.java:302)
SCENE8_LIGHT = ((123.0, 554.0, 147.0), (300.0, 0.0, 0.0), (0.0, 0.0, 265.0))
# the moving sphere (400,400,200) -> (500,400,200), r 50 (Scene.java:304-307): swept, excluded
SCENE8_MOVING = ((400.0, 400.0, 200.0), (500.0, 400.0, 200.0), 50.0)
# the 1000-sphere cluster: centres in [0,165)^3 + (-100, 270, 395), r 10 (Scene.java:329-334)
SCENE8_CLUSTER = ((-110.0, 260.0, 385.0), (75.0, 445.0, 570.0))
GROUND_TOP = 101.0   # the ground boxes reach y = 1 + 100*Math.random()
# Scene.java:44-104 (scene 0, bouncingSpheres): the three fixed spheres of radius 1; the
# random small spheres (r 0.2 at y 0.2, some moving up by up to 0.5) stay below y = 0.9
SCENE0_SPHERES = {
    "glass": ((0.0, 1.0, 0.0), 1.0),        # Dielectric(1.5)
    "diffuse": ((-4.0, 1.0, 0.0), 1.0),     # Lambertian(0.4, 0.2, 0.1)
    "metal": ((4.0, 1.0, 0.0), 1.0),        # Metal(0.7, 0.6, 0.5; fuzz 0)
}
SCENE0_SMALL_TOP = 0.9


def camera_rays(camera, width, height):
    """Pixel-centre rays (origin, unnormalized direction) of the UBO camera:
    get_norm_coord (compute.glsl:268-283) without the jitter."""
    cam = np.asarray(camera, np.float64)
    pos, up_left, du, dv = cam[4:7], cam[8:11], cam[12:15], cam[16:19]
    xs, ys = np.meshgrid(np.arange(width, dtype=np.float64), np.arange(height, dtype=np.float64))
    target = up_left + xs[..., None] * du + ys[..., None] * dv
    return pos, target - pos


def _sphere_t(o, d, c, r):
    oc = o - np.asarray(c)
    a = (d * d).sum(-1)
    hb = (d * oc).sum(-1)
    cc = (oc * oc).sum() - r * r
    disc = hb * hb - a * cc
    t = np.full(a.shape, np.inf)
    ok = disc >= 0
    sq = np.sqrt(np.where(ok, disc, 0.0))
    t0 = (-hb - sq) / a
    t1 = (-hb + sq) / a
    t = np.where(ok & (t0 > 1e-3), t0, np.where(ok & (t1 > 1e-3), t1, np.inf))
    return t


def _sphere_near(o, d, c, r, margin):
    """True where the ray passes within r + margin of the centre (t > 0)."""
    oc = np.asarray(c) - o
    a = (d * d).sum(-1)
    tc = (d * oc).sum(-1) / a
    closest = oc - tc[..., None] * d
    dist = np.sqrt((closest * closest).sum(-1))
    return (dist < r + margin) & (tc > 0)


def _aabb_t(o, d, lo, hi):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t0 = (np.asarray(lo) - o) * inv
        t1 = (np.asarray(hi) - o) * inv
    tmin = np.nanmax(np.minimum(t0, t1), axis=-1)
    tmax = np.nanmin(np.maximum(t0, t1), axis=-1)
    hit = (tmax >= np.maximum(tmin, 0.0))
    return np.where(hit, np.maximum(tmin, 0.0), np.inf)


def scene8_regions(camera, width, height, erode=2):
    """{name: bool[H, W]} for the light quad and the five deterministic spheres,
    each pixel assigned to the first deterministic object on its pixel-centre ray
    and kept only when no excluded geometry can come first (ground boxes below
    y = GROUND_TOP + margin, the cluster box, the moving sphere's sweep) and
    every pixel within `erode` pixels has the same first object (no silhouettes:
    the jittered samples of an edge pixel see both sides)."""
    o, d = camera_rays(camera, width, height)
    names = list(SCENE8_SPHERES) + ["light"]
    ts = [_sphere_t(o, d, c, r) for c, r in SCENE8_SPHERES.values()]
    q, u, v = (np.asarray(x) for x in SCENE8_LIGHT)
    n = np.cross(u, v)
    denom = (d * n).sum(-1)
    with np.errstate(divide="ignore", invalid="ignore"):
        tq = (n @ q - n @ o) / denom
    p = o + tq[..., None] * d - q
    al, be = p[..., 0] / u[0], p[..., 2] / v[2]
    ts.append(np.where((tq > 1e-3) & (al >= 0) & (al <= 1) & (be >= 0) & (be <= 1), tq, np.inf))
    T = np.stack(ts)
    first = np.argmin(T, axis=0)
    tbest = np.min(T, axis=0)
    ok = np.isfinite(tbest)
    hit_y = o[1] + tbest * d[..., 1]
    # excluded geometry in front: the ground boxes' slab y < GROUND_TOP (+ margin), the cluster, the sweep
    with np.errstate(divide="ignore", invalid="ignore"):
        t_ground = np.where(d[..., 1] < 0, (GROUND_TOP + 5.0 - o[1]) / d[..., 1], np.inf)
    ok &= ~(t_ground < tbest) & (hit_y > GROUND_TOP + 5.0)
    lo, hi = SCENE8_CLUSTER
    ok &= ~(_aabb_t(o, d, np.asarray(lo) - 5.0, np.asarray(hi) + 5.0) < tbest)
    c0, c1, rm = SCENE8_MOVING
    for k in range(11):
        c = np.asarray(c0) + (np.asarray(c1) - np.asarray(c0)) * (k / 10.0)
        ok &= ~(_sphere_near(o, d, c, rm, 8.0) & (_sphere_t(o, d, c, rm + 8.0) < tbest))
    lab = np.where(ok, first, -1)
    # erode: every neighbour within `erode` pixels has the same label
    keep = lab >= 0
    for dy in range(-erode, erode + 1):
        for dx in range(-erode, erode + 1):
            sh = np.full_like(lab, -2)
            ys = slice(max(0, dy), height + min(0, dy))
            yd = slice(max(0, -dy), height + min(0, -dy))
            xs = slice(max(0, dx), width + min(0, dx))
            xd = slice(max(0, -dx), width + min(0, -dx))
            sh[yd, xd] = lab[ys, xs]
            keep &= sh == lab
    return {nm: keep & (lab == i) for i, nm in enumerate(names)}


def scene0_regions(camera, width, height, erode=3):
    """{name: bool[H, W]} for scene 0's three fixed spheres: the first of them on the
    pixel-centre ray, hit above y = SCENE0_SMALL_TOP + 0.1 (the camera looks down from
    y = 2, so such a ray never crossed the random small spheres' layer first), every pixel
    within `erode` pixels the same (defocus blur and jitter see both sides of an edge)."""
    o, d = camera_rays(camera, width, height)
    names = list(SCENE0_SPHERES)
    T = np.stack([_sphere_t(o, d, c, r) for c, r in SCENE0_SPHERES.values()])
    first = np.argmin(T, axis=0)
    tbest = np.min(T, axis=0)
    ok = np.isfinite(tbest) & (o[1] + tbest * d[..., 1] > SCENE0_SMALL_TOP + 0.1)
    lab = np.where(ok, first, -1)
    keep = lab >= 0
    for dy in range(-erode, erode + 1):
        for dx in range(-erode, erode + 1):
            sh = np.full_like(lab, -2)
            ys = slice(max(0, dy), height + min(0, dy))
            yd = slice(max(0, -dy), height + min(0, -dy))
            xs = slice(max(0, dx), width + min(0, dx))
            xd = slice(max(0, -dx), width + min(0, -dx))
            sh[yd, xd] = lab[ys, xs]
            keep &= sh == lab
    return {nm: keep & (lab == i) for i, nm in enumerate(names)}


def block_grid(mask, block):
    """Blocks of `block` x `block` pixels lying wholly inside `mask`: list of (y0, x0)."""
    h, w = mask.shape
    out = []
    for y0 in range(0, h - block + 1, block):
        for x0 in range(0, w - block + 1, block):
            if mask[y0:y0 + block, x0:x0 + block].all():
                out.append((y0, x0))
    return out


def block_means(rgb, blocks, block):
    return np.array([rgb[y:y + block, x:x + block].reshape(-1, rgb.shape[-1]).mean(0) for y, x in blocks])
