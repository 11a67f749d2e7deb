"""Build-defined adversarial scenes for the parity tests (test infrastructure).

They aim rays at what the kernel's exactness shortcuts could get
wrong, through the reference's own builder calls (rtamd.SceneBuilder) and a
camera block written directly so that camera rays are exact binary fractions:
with recip_sqrt_spp = 0 the stratified jitter vanishes (random.glsl:82-100:
(col + 0.5) * 0 and (rand() - 0.5) * 0) and pixel (x, y)'s ray is
    d = up_left + du * x + dv * y - (du + dv) / 2 - camera_pos
(compute.glsl:268-296), computed exactly for the grids below.  The reference's
hit tests they target (hitting.glsl:90-146):
  * box edges and corners hit exactly (alpha / beta at 0 and 1), canonical and
    y-rotated boxes;
  * grazing faces: |dot(n, d)| around, at and just below the 1e-8 cut;
  * plane t at, just below and just above tmin = 0.001 (inclusive for quads,
    strict for spheres);
  * scenes scaled so their extent sits just inside / just past 2^20, where the
    shared-reciprocal division stops applying (rt_capi.hip fd_coord);
  * BVHs beyond the round-2 link-format cap of 2047 nodes, one in LDS (~4000
    nodes) and one that needs the two-level walk (~9000 nodes);
  * walks that start past the root's right spine (rt_kernel.hip spine_entry): ray
    origins just inside the spine's box, where its face is 0.0008 / 0.0019 / 0.01 ahead
    (the reference's slab test misses / hits just past tmin / hits), with direction
    components up to 2 so that the entry's margin 0.00125 max|d| falls inside the pixel
    grid; and near an edge of the box.
Secondary bounces add random rays around the same geometry.
"""
import numpy as np

import rtamd
from rtamd.scene import SceneBuilder

F32 = np.float32


def grid_camera(origin, up_left, du, dv):
    """The 28-float camera block (rt_camera_ubo) of an exact ray grid."""
    u = np.zeros(28, F32)
    u[0:4] = [2.0, 2.0, 1.0, 0.0]           # viewport w/h, aspect, defocus_angle = 0 (no disk)
    u[4:7], u[8:11], u[12:15], u[16:19] = origin, up_left, du, dv
    return u


EXACT = (1.0, 0.0)   # (sqrt_spp, recip_sqrt_spp): no jitter


class Case:
    """One adversarial configuration: a scene, its uniforms and render size."""

    def __init__(self, name, scene, frames=3, depth=4, uniforms=EXACT, spp=None, expect=None):
        self.name, self.scene, self.frames, self.depth = name, scene, frames, depth
        self.uniforms = uniforms if spp is None else rtamd.spp_uniforms(spp)
        self.expect = expect or {}   # rt_debug_last_launch fields the default render must show


def _materials(b):
    white = b.lambertian(b.solid(0.73, 0.73, 0.73))
    red = b.lambertian(b.solid(0.65, 0.05, 0.05))
    light = b.diffuse_light(6, 6, 6)
    return white, red, light


def edges(rotated=False, W=64, H=48):
    """Boxes whose edges and corners camera rays hit exactly: d = (-2 + x/16, 1.5 - y/16, -1)
    meets the front face z = -4 of box 1 at (4 d.x, 4 d.y) -- its edges x = +-2 at pixel
    columns 24 and 56 -- and y = +-1 (rows 20 and 28); box 2's front face z = -8 at
    multiples of 1/2.  rotated: box 2 and 3 turned about y (the general box test)."""
    b = SceneBuilder(seed=1)
    white, red, light = _materials(b)
    b.add(b.box((-2, -1, -8), (2, 1, -4), white))
    if rotated:
        b.add(b.box((0, 0, 0), (3, 2.5, 3), red, translation=(-1.5, -3, -11), rotation=(0, F32(0.2617994), 0)))
        b.add(b.box((0, 0, 0), (2, 2, 2), white, translation=(1, 0.5, -14), rotation=(0, F32(-0.5235988), 0)))
    else:
        b.add(b.box((-1.5, -3, -12), (3, -0.5, -8), red))
        b.add(b.box((1, 0.5, -16), (3.5, 3, -12), white))
    b.add(b.sphere((-1, 1.75, -6), 0.75, b.metal(b.solid(0.8, 0.8, 0.9), 0.25)))
    lq = b.add(b.quad((-3, 4, -12), (6, 0, 0), (0, 0, 8), light))
    b.add_light(lq)
    b.add(b.box((-6, -5, -20), (6, -4, 2), white))   # a floor slab under everything
    b.camera(background=(0.2, 0.25, 0.3))
    s = b.finish(W, H)
    s.override_camera(grid_camera((0, 0, 0), (-2 + 1 / 32, 1.5 - 1 / 32, -1), (1 / 16, 0, 0), (0, -1 / 16, 0)))
    return s


def grazing(mode, W=64, H=48):
    """A box whose top face y = top meets camera rays at |dot(n, d)| = |d.y| near 1e-8:
    'grid'  : d.y from ~-1.4e-8 to 3e-8 in steps of 2^-30, origin 1.5 * 2^-24 above y = 0;
    'cut'   : every d.y = -1e-8f exactly (the cut is |denom| < 1e-8: still tested);
    'below' : every d.y = -(the float below 1e-8) (skipped)."""
    b = SceneBuilder(seed=1)
    white, red, light = _materials(b)
    top = 0.0 if mode == "grid" else float(F32(-8e-8))
    b.add(b.box((-4, -2, -12), (4, top, -4), white))
    b.add(b.box((-1, top, -20), (1, 0.5, -14), red))
    lq = b.add(b.quad((-3, 3, -10), (6, 0, 0), (0, 0, 4), light))
    b.add_light(lq)
    b.camera(background=(0.3, 0.3, 0.3))
    s = b.finish(W, H)
    if mode == "grid":
        oy = 1.5 * 2.0 ** -24
        origin, ul, dv = (0, oy, 0), (-2 + 1 / 32, oy + 2.0 ** -25, -1), (0, -(2.0 ** -30), 0)
    else:
        dy = F32(1e-8) if mode == "cut" else np.nextafter(F32(1e-8), F32(0))
        origin, ul, dv = (0, 0, 0), (-2 + 1 / 32, -dy, -1), (0, 0, 0)
    s.override_camera(grid_camera(origin, ul, (1 / 16, 0, 0), dv))
    return s


def tmin(mode, W=64, H=48):
    """Plane t at tmin = 0.001 (hitting.glsl: quads accept t in [tmin, max], spheres need
    tmin < root): a box's front face z = 0 seen from z = 0.001f (t = 0.001f exactly for
    every camera ray), from the float below (t < tmin: the face is skipped, the ray goes on
    inside the box) and above; 'sphere': a sphere whose surface is 0.001f ahead."""
    b = SceneBuilder(seed=1)
    white, red, light = _materials(b)
    if mode == "sphere":
        b.add(b.sphere((0, 0, -1), 1.0, white))
        b.add(b.box((-3, -3, -6), (3, 3, -5), red))
    else:
        b.add(b.box((-2, -1, -2), (2, 1, 0), white))
        b.add(b.box((-3, -3, -6), (3, 3, -5), red))
    lq = b.add(b.quad((-2, 2.5, -4), (4, 0, 0), (0, 0, 3), light))
    b.add_light(lq)
    b.camera(background=(0.3, 0.3, 0.3))
    s = b.finish(W, H)
    z0 = F32(0.001)
    z = {"at": z0, "below": np.nextafter(z0, F32(0)), "above": np.nextafter(z0, F32(1)), "sphere": z0}[mode]
    s.override_camera(grid_camera((0, 0, z), (-2 + 1 / 32, 1.5 - 1 / 32, z - 1), (1 / 16, 0, 0), (0, -1 / 16, 0)))
    return s


def extent(dist, W=64, H=48, S=16.0):
    """The edges scene at scale S (box edges up to 352, so every face's delta stays within
    the shared-reciprocal regime's 2^20) moved `dist` from the origin along -z: the scene's
    extent (max |coordinate| of records and camera) is about dist."""
    c = np.array([0.0, 0.0, -dist], F32)
    p = lambda x, y, z: tuple(float(v) for v in (c + F32(S) * np.array([x, y, z], F32)))  # noqa: E731
    b = SceneBuilder(seed=1)
    white, red, light = _materials(b)
    b.add(b.box(p(-2, -1, -8), p(2, 1, -4), white))
    b.add(b.box(p(-1.5, -3, -12), p(3, -0.5, -8), red))
    b.add(b.box(p(-6, -5, -20), p(6, -4, 2), white))
    lq = b.add(b.quad(p(-3, 4, -12), (6 * S, 0, 0), (0, 0, 8 * S), light))
    b.add_light(lq)
    b.camera(background=(0.3, 0.3, 0.3))
    s = b.finish(W, H)
    ul = np.array([-2 + 1 / 32, 1.5 - 1 / 32, -1], F32) * F32(S)
    s.override_camera(grid_camera(c, c + ul, (S / 16, 0, 0), (0, -S / 16, 0)))
    return s


def sphere_cloud(n, seed, W=64, H=48, boxes=True):
    """n small spheres in a cloud (+ a few canonical boxes): a BVH of about n nodes."""
    rng = np.random.default_rng(seed)
    b = SceneBuilder(seed=1)
    white, red, light = _materials(b)
    glass = b.dielectric(1.5)
    mats = [white, red, glass]
    pts = rng.uniform(-1, 1, (n, 3)).astype(F32) * F32([6, 4, 6]) + F32([0, 0, -14])
    for k in range(n):
        b.add(b.sphere(tuple(float(v) for v in pts[k]), 0.12, mats[k % 3]))
    if boxes:
        for k in range(8):
            x0 = -8 + 2 * k
            b.add(b.box((x0, -6, -20), (x0 + 1.5, -5 + 0.25 * k, -8), white))
    lq = b.add(b.quad((-4, 6, -18), (8, 0, 0), (0, 0, 8), light))
    b.add_light(lq)
    b.camera(look_from=(0, 1, 2), look_at=(0, 0, -14), vfov=60, background=(0.5, 0.6, 0.8))
    return b.finish(W, H)


def spine_box(scene):
    """The intersection of the boxes on the threaded BVH's right spine (root, its right
    child, ... to the first leaf): what rt_capi.hip plan_spine intersects."""
    import ctypes
    L = rtamd.amd()
    bvh = scene.buffers[1]
    raw = np.frombuffer(bvh.data if hasattr(bvh, "data") else bvh, np.uint8)
    dn = np.dtype([("box", "<f4", (6,)), ("meta", "<u4"), ("prims", "<u4")])
    n = ctypes.c_int()
    assert L.rt_debug_threaded_bvh(raw.ctypes.data, raw.nbytes, None, 0, ctypes.byref(n)) == 0
    out = np.zeros(n.value, dn)
    assert L.rt_debug_threaded_bvh(raw.ctypes.data, raw.nbytes, out.ctypes.data, out.nbytes, ctypes.byref(n)) == 0
    lo, hi = np.full(3, -np.inf, F32), np.full(3, np.inf, F32)
    for nd in out:
        bx = nd["box"]
        lo = np.maximum(lo, bx[0::2])
        hi = np.minimum(hi, bx[1::2])
        if (int(nd["meta"]) >> 16) & 0xF:
            break
    return lo, hi, len(out)


def spine(delta, corner=False, W=64, H=48):
    """Scene 8's shape in small: a fog whose boundary sphere (r 50) is the BVH's largest
    object, so it sits in the right-most leaf and every box on the right spine contains it,
    around a cluster of small spheres and boxes; dense (2000), so rays leaving the camera
    scatter within ~0.0005 and the next walks start from origins just inside the faces too.
    The camera sits `delta` inside the
    spine box's +x face on the x axis (corner: also delta below its +y face) and
    looks along +x: d = (1, y, z), |y|, |z| <= 2, so the face is delta / 1 ahead."""
    rng = np.random.default_rng(5)
    b = SceneBuilder(seed=1)
    white, red, light = _materials(b)
    fog = b.sphere((0, 0, 0), 50.0, b.dielectric(1.5))
    b.add(b.constant_medium(fog, 2000.0, b.isotropic(b.solid(0.9, 0.9, 0.9))))   # scatters within ~0.0005
    for k in range(40):
        c = tuple(float(v) for v in rng.uniform(-8, 8, 3).astype(F32))
        b.add(b.sphere(c, 0.7, white if k % 2 else red))
    for k in range(4):
        b.add(b.box((-9 + 4 * k, -10, -9), (-7 + 4 * k, -9 + k, 9), white))
    lq = b.add(b.quad((-5, 12, -5), (10, 0, 0), (0, 0, 10), light))
    b.add_light(lq)
    b.camera(look_from=(0, 0, 30), look_at=(0, 0, 0), vfov=40, background=(0.2, 0.25, 0.3))
    s = b.finish(W, H)
    lo, hi, _ = spine_box(s)
    # on the x axis: the fog's sphere touches the box's face there, so the camera is delta
    # inside the fog too and rays leaving it scatter (or not) right at the face
    o = np.array([hi[0] - F32(delta), 0, 0], F32)
    if corner:   # and delta below the +y face (outside the fog, in the box's edge region)
        o[1] = hi[1] - F32(delta)
    s.override_camera(grid_camera(tuple(float(v) for v in o), tuple(float(v) for v in o + F32([1, 2, -2])),
                                  (0, 0, F32(1 / 16)), (0, -F32(1 / 12), 0)))
    return s


def cases():
    """The configurations, each with what its default launch must show."""
    big = 2 ** 20
    return [
        Case("edges", edges(), expect={"box_records": 3}),
        Case("edges_jitter", edges(), spp=16, frames=4),
        Case("edges_rotated", edges(rotated=True), expect={"box_records": 2}),
        Case("grazing_grid", grazing("grid")),
        Case("grazing_cut", grazing("cut")),
        Case("grazing_below", grazing("below")),
        Case("tmin_at", tmin("at")),
        Case("tmin_below", tmin("below")),
        Case("tmin_above", tmin("above")),
        Case("tmin_sphere", tmin("sphere")),
        Case("extent_inside_2^20", extent(0.95 * big), expect={"fastdiv": 1, "pretest": 1}),
        Case("extent_past_2^20", extent(1.1 * big), expect={"fastdiv": 0, "pretest": 1}),
        Case("bvh_4k_lds", sphere_cloud(4000, 4), depth=3, frames=2, expect={"shape": 2, "block": 1024}),
        Case("bvh_9k_two_level", sphere_cloud(9000, 9), depth=3, frames=2, expect={"shape": 5, "block": 1024}),
        Case("spine_face_0.0008", spine(0.0008)),
        Case("spine_face_0.0019", spine(0.0019)),
        Case("spine_face_0.01", spine(0.01)),
        Case("spine_edge_0.0019", spine(0.0019, corner=True)),
        Case("spine_jitter", spine(0.0019), spp=16, frames=4),
    ]
