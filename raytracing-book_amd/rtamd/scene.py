"""Python face of the host scene builder (mirror of the reference's Scene API).

``Scene(scene_id, width, height, seed)`` corresponds to the reference's
``new Scene(sceneID, initImageWidth, initImageHeight, computeProgram)``
(J/draw/Scene.java:15-35): it builds one of the built-in scenes 0-8 (plus the
build-defined scene 9), constructs the BVH and packs every SSBO exactly as
``RaytraceModel.putModelsToProgram`` does.  Instead of uploading to OpenGL it
exposes the bytes, which ``RenderContext.upload_scene`` hands to rt.h.
"""
import ctypes

import numpy as np

from . import _lib

SCENE_NAMES = {
    0: "bouncingSpheres (Book 1 final)",
    1: "checkerSpheres",
    2: "earth",
    3: "perlinSpheres",
    4: "quads",
    5: "simpleLight",
    6: "cornellBox (Book 3 final)",
    7: "cornellSmoke",
    8: "finalScene (Book 2 final)",
    9: "three spheres (build-defined, SURVEY C1)",
}

# rt.h bindings / record sizes (rt_types.h)
BIND_SPHERES, BIND_BVH, BIND_QUADS, BIND_MEDIA, BIND_BOXES, BIND_LIGHTS = range(6)
RECORD_BYTES = {BIND_SPHERES: 48, BIND_BVH: 32, BIND_QUADS: 80, BIND_MEDIA: 20, BIND_BOXES: 480, BIND_LIGHTS: 4}
TEX_RGB8, TEX_RGBA8, TEX_R32F = 1, 2, 3


class Texture:
    __slots__ = ("slot", "format", "width", "height", "data")

    def __init__(self, slot, fmt, w, h, data):
        self.slot, self.format, self.width, self.height, self.data = slot, fmt, w, h, data


class Scene:
    """A built scene: SSBO bytes, textures, camera UBO and uniforms."""

    def __init__(self, scene_id, width, height, seed=1, asset_dir=None, _handle=None):
        L = _lib.scene_lib()
        if _handle is None:
            h = ctypes.c_void_p()
            ad = (asset_dir or _lib.ASSET_DIR).encode()
            rc = L.rts_build(int(scene_id), int(width), int(height), ctypes.c_uint64(seed), ad, ctypes.byref(h))
            if rc != 0:
                raise ValueError(L.rts_last_error().decode())
        else:
            h = _handle
        self._h = h
        self.scene_id = int(scene_id)
        self.seed = seed
        self._refresh()

    def override_camera(self, ubo):
        """Replace the 28-float camera block (tests aim exact rays with it)."""
        ubo = np.asarray(ubo, np.float32).ravel()
        assert ubo.size == 28
        self.camera = ubo.copy()

    def _refresh(self):
        L = _lib.scene_lib()
        info = _lib.RtsInfo()
        L.rts_get_info(self._h, ctypes.byref(info))
        self.info = {k: getattr(info, k) for k, _ in _lib.RtsInfo._fields_ if k != "background"}
        self.background = np.array(info.background[:], dtype=np.float32)
        self.width, self.height = info.width, info.height
        self.buffers = {}
        for b in range(6):
            p, n = ctypes.c_void_p(), ctypes.c_size_t()
            L.rts_get_buffer(self._h, b, ctypes.byref(p), ctypes.byref(n))
            self.buffers[b] = ctypes.string_at(p, n.value) if n.value else b""
        self.textures = []
        for s in range(info.n_textures):
            f, w, hh = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            p, n = ctypes.c_void_p(), ctypes.c_size_t()
            L.rts_get_texture(self._h, s, ctypes.byref(f), ctypes.byref(w), ctypes.byref(hh), ctypes.byref(p),
                              ctypes.byref(n))
            self.textures.append(Texture(s, f.value, w.value, hh.value, ctypes.string_at(p, n.value)))
        cam = (ctypes.c_float * 28)()
        L.rts_get_camera(self._h, cam)
        self.camera = np.array(cam[:], dtype=np.float32)

    def set_image_size(self, width, height):
        """Scene.updateCamera (Scene.java:37-41)."""
        _lib.scene_lib().rts_set_image_size(self._h, int(width), int(height))
        self._refresh()

    def close(self):
        if self._h:
            _lib.scene_lib().rts_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def spp_uniforms(spp):
    """RaytraceExecutor.setSamplePerPixel: ((float)Math.sqrt(spp), 1f/sqrtSpp)."""
    a, b = ctypes.c_float(), ctypes.c_float()
    _lib.scene_lib().rts_spp_uniforms(int(spp), ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def tonemap_rgb8(rgba):
    """Texture.saveAsPNG pixel pipeline (Texture.java:93-99) -> uint8 [H,W,3]."""
    rgba = np.ascontiguousarray(rgba, dtype=np.float32)
    h, w = rgba.shape[:2]
    out = np.empty((h, w, 3), dtype=np.uint8)
    rc = _lib.scene_lib().rts_tonemap_rgb8(rgba.ctypes.data_as(_lib.c_float_p), w, h,
                                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    if rc:
        raise ValueError("tonemap failed")
    return out


def save_png(rgba, path):
    """Texture.saveAsPNG (Texture.java:89-120)."""
    rgba = np.ascontiguousarray(rgba, dtype=np.float32)
    h, w = rgba.shape[:2]
    rc = _lib.scene_lib().rts_save_png(rgba.ctypes.data_as(_lib.c_float_p), w, h, str(path).encode())
    if rc:
        raise IOError(f"saving {path} failed ({rc})")


def decode_image(path):
    """ImageTexture.create's read (ImageTexture.java:22-85: ImageIO.read + getRGB) of a JPEG,
    PNG or P6 PPM file -> uint8 [H, W, 3 or 4], row 0 = top (rt_scene.h rts_decode_image).
    Raises ValueError where the reference throws (unsupported component counts)."""
    L = _lib.scene_lib()
    w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    p = str(path).encode()
    if L.rts_decode_image(p, ctypes.byref(w), ctypes.byref(h), ctypes.byref(c), None, 0):
        raise ValueError(L.rts_decode_last_error().decode())
    out = np.empty((h.value, w.value, c.value), dtype=np.uint8)
    if L.rts_decode_image(p, ctypes.byref(w), ctypes.byref(h), ctypes.byref(c),
                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.size):
        raise ValueError(L.rts_decode_last_error().decode())
    return out


MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_ISOTROPIC = range(5)


class SceneBuilder:
    """The reference's scene-building calls (Scene.java) on an empty world (rt_scene.h rts_new).

    Textures and materials are shared objects (their ids / handles), models are
    created, then added (RaytraceModel.addModel / addLight); ``finish(w, h)``
    builds the BVH, packs the records and returns a :class:`Scene`::

        b = SceneBuilder(seed=1)
        white = b.lambertian(b.solid(0.73, 0.73, 0.73))
        b.add(b.box((0, 0, 0), (1, 2, 1), white))
        b.camera(look_from=(0, 1, 5), look_at=(0, 1, 0), vfov=40)
        scene = b.finish(64, 48)
    """

    def __init__(self, seed=1, asset_dir=None):
        self._L = _lib.scene_lib()
        self._h = ctypes.c_void_p()
        ad = (asset_dir or _lib.ASSET_DIR).encode()
        self._check(self._L.rts_new(ctypes.c_uint64(seed), ad, ctypes.byref(self._h)))
        self.seed = seed
        self._done = False

    def _check(self, rc):
        if rc != 0:
            raise ValueError(self._L.rts_last_error().decode())

    def _out(self, fn, *args):
        if self._done:
            raise ValueError("the scene was already finished (rts_finish)")
        v = ctypes.c_int()
        self._check(fn(self._h, *args, ctypes.byref(v)))
        return v.value

    @staticmethod
    def _v(x):
        return (ctypes.c_float * 3)(*[float(c) for c in x]) if x is not None else None

    # textures (packed ids)
    def solid(self, r, g, b):
        return self._out(self._L.rts_solid_texture, ctypes.c_float(r), ctypes.c_float(g), ctypes.c_float(b))

    def checker(self, c1, c2, scale):
        return self._out(self._L.rts_checker_texture, self._v(c1), self._v(c2), ctypes.c_float(scale))

    def perlin(self, scale):
        return self._out(self._L.rts_perlin_texture, ctypes.c_float(scale))

    def image(self, asset_name, shift_x=0, shift_y=0):
        return self._out(self._L.rts_image_texture, asset_name.encode(), int(shift_x), int(shift_y))

    # materials (handles)
    def material(self, kind, texture=0, param=0.0, emit=None):
        return self._out(self._L.rts_material, int(kind), int(texture), ctypes.c_float(param), self._v(emit))

    def lambertian(self, tex):
        return self.material(MAT_LAMBERTIAN, tex)

    def metal(self, tex, fuzz):
        return self.material(MAT_METAL, tex, fuzz)

    def dielectric(self, ior):
        return self.material(MAT_DIELECTRIC, 0, ior)

    def diffuse_light(self, r, g, b):
        return self.material(MAT_DIFFUSE_LIGHT, 0, 0.0, (r, g, b))

    def isotropic(self, tex):
        return self.material(MAT_ISOTROPIC, tex)

    # models (handles)
    def sphere(self, center, radius, mat, center2=None):
        return self._out(self._L.rts_sphere, self._v(center), self._v(center2), ctypes.c_float(radius), int(mat))

    def quad(self, q, u, v, mat):
        return self._out(self._L.rts_quad, self._v(q), self._v(u), self._v(v), int(mat))

    def box(self, a, b, mat, translation=None, rotation=None):
        return self._out(self._L.rts_box, self._v(a), self._v(b), self._v(translation), self._v(rotation), int(mat))

    def constant_medium(self, boundary, density, mat):
        return self._out(self._L.rts_constant_medium, int(boundary), ctypes.c_float(density), int(mat))

    def add(self, model):
        self._check(self._L.rts_add_model(self._h, int(model)))
        return model

    def add_light(self, model):
        self._check(self._L.rts_add_light(self._h, int(model)))
        return model

    def camera(self, look_from=(0, 0, 0), look_at=(0, 0, -1), vup=(0, 1, 0), vfov=90.0, defocus_angle=0.0,
               focus_dist=10.0, background=(0, 0, 0)):
        p = _lib.RtsCamera()
        p.look_from[:] = [float(c) for c in look_from]
        p.look_at[:] = [float(c) for c in look_at]
        p.vup[:] = [float(c) for c in vup]
        p.vfov, p.defocus_angle, p.focus_dist = float(vfov), float(defocus_angle), float(focus_dist)
        p.background[:] = [float(c) for c in background]
        self._check(self._L.rts_camera(self._h, ctypes.byref(p)))

    def finish(self, width, height):
        self._check(self._L.rts_finish(self._h, int(width), int(height)))
        self._done = True
        sc = Scene(-1, width, height, seed=self.seed, _handle=self._h)
        self._h = None
        return sc

    def __del__(self):
        try:
            if self._h and not self._done:
                self._L.rts_free(self._h)
        except Exception:
            pass
