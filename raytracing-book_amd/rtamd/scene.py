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

    def __init__(self, scene_id, width, height, seed=1, asset_dir=None):
        L = _lib.scene_lib()
        h = ctypes.c_void_p()
        ad = (asset_dir or _lib.ASSET_DIR).encode()
        rc = L.rts_build(int(scene_id), int(width), int(height), ctypes.c_uint64(seed), ad, ctypes.byref(h))
        if rc != 0:
            raise ValueError(L.rts_last_error().decode())
        self._h = h
        self.scene_id = int(scene_id)
        self.seed = seed
        self._refresh()

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
