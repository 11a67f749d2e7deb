"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (liboracle.so).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Never used by the product path (raytracing-book_amd/).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_L = None


class OracleSceneDesc(ctypes.Structure):
    _fields_ = [
        ("buf", ctypes.c_void_p * 6),
        ("nbytes", ctypes.c_size_t * 6),
        ("tex_format", ctypes.c_int * 8),
        ("tex_w", ctypes.c_int * 8),
        ("tex_h", ctypes.c_int * 8),
        ("tex", ctypes.c_void_p * 8),
        ("camera", ctypes.c_float * 28),
        ("max_depth", ctypes.c_int),
        ("background", ctypes.c_float * 3),
        ("sqrt_spp", ctypes.c_float),
        ("recip_sqrt_spp", ctypes.c_float),
    ]


COUNTER_FIELDS = ["samples", "bounces", "node_visits", "sphere_tests", "quad_tests", "box_tests", "medium_tests",
                  "rand_calls", "framebuffer_bytes", "node_bytes", "prim_bytes", "material_bytes", "texel_bytes",
                  "light_bytes"]


class OracleCounters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in COUNTER_FIELDS]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        fp = ctypes.POINTER(ctypes.c_float)
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [ctypes.POINTER(OracleSceneDesc), ctypes.c_int, ctypes.c_int, fp, ctypes.c_int,
                                    ctypes.c_int, fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(OracleCounters)]
        L.oracle_set_thread_cpus.restype = None
        L.oracle_set_thread_cpus.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.oracle_get_sphere_uv.argtypes = [ctypes.c_float] * 3 + [fp, fp]
        L.oracle_rand_sequence.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int, fp]
        L.oracle_eval_builtin.argtypes = [ctypes.c_int, fp, fp, fp, ctypes.c_int]
        L.oracle_perlin_turb.restype = ctypes.c_float
        L.oracle_perlin_turb.argtypes = [fp, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.oracle_hit_sphere.argtypes = [ctypes.c_void_p, ctypes.c_float, fp, fp, ctypes.c_float, ctypes.c_float,
                                        fp, fp, fp, ctypes.POINTER(ctypes.c_int)]
        L.oracle_hit_quad.argtypes = [ctypes.c_void_p, fp, fp, ctypes.c_float, ctypes.c_float, fp, fp, fp,
                                      ctypes.POINTER(ctypes.c_int)]
        L.oracle_hit_aabb.argtypes = [fp, fp, fp, ctypes.c_float, ctypes.c_float]
        _L = L
    return _L


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class OracleScene:
    """Keeps the scene bytes alive and describes them to the oracle."""

    def __init__(self, scene, max_depth=5, spp=1, background=None, uniforms=None):
        from rtamd.scene import spp_uniforms   # host-side uniform helper
        self.keep = []
        d = OracleSceneDesc()
        for b in range(6):
            data = scene.buffers[b]
            if data:
                cb = ctypes.create_string_buffer(data, len(data))
                self.keep.append(cb)
                d.buf[b] = ctypes.cast(cb, ctypes.c_void_p)
            d.nbytes[b] = len(data)
        for t in scene.textures:
            cb = ctypes.create_string_buffer(t.data, len(t.data))
            self.keep.append(cb)
            d.tex[t.slot] = ctypes.cast(cb, ctypes.c_void_p)
            d.tex_format[t.slot], d.tex_w[t.slot], d.tex_h[t.slot] = t.format, t.width, t.height
        for i in range(28):
            d.camera[i] = float(scene.camera[i])
        d.max_depth = max_depth
        bg = scene.background if background is None else background
        for i in range(3):
            d.background[i] = float(bg[i])
        d.sqrt_spp, d.recip_sqrt_spp = spp_uniforms(spp) if uniforms is None else (float(uniforms[0]),
                                                                                   float(uniforms[1]))
        self.desc = d
        self.width, self.height = scene.width, scene.height


def render(oscene, rand_factors, first_frame=1, image=None, rank=0, world=1, stripe_rows=16, nthreads=0,
           counters=False):
    """Render frames first_frame.. into `image` ([H, W, 4] float32, zero-init)."""
    L = lib()
    W, H = oscene.width, oscene.height
    if image is None:
        image = np.zeros((H, W, 4), dtype=np.float32)
    if image.shape != (H, W, 4) or image.dtype != np.float32 or not image.flags.c_contiguous:
        raise ValueError(f"oracle image must be a contiguous float32 [{H}, {W}, 4] array (full size, any rank)")
    rf = np.ascontiguousarray(rand_factors, dtype=np.float32)
    cnt = OracleCounters() if counters else None
    rc = L.oracle_render(ctypes.byref(oscene.desc), W, H, _fp(image), int(first_frame), int(rf.size), _fp(rf),
                         rank, world, stripe_rows, nthreads, ctypes.byref(cnt) if cnt is not None else None)
    if rc != 0:
        raise RuntimeError(f"oracle_render failed ({rc})")
    if counters:
        return image, {n: getattr(cnt, n) for n in COUNTER_FIELDS}
    return image


def set_thread_cpus(cpus):
    """Pin render()'s worker i to CPU cpus[i % len(cpus)]; None or [] unpins."""
    cpus = list(cpus or [])
    arr = (ctypes.c_int * max(1, len(cpus)))(*cpus)
    lib().oracle_set_thread_cpus(arr, len(cpus))


def sphere_uv(x, y, z):
    u, v = ctypes.c_float(), ctypes.c_float()
    lib().oracle_get_sphere_uv(x, y, z, ctypes.byref(u), ctypes.byref(v))
    return u.value, v.value


def rand_sequence(px, py, f, n):
    out = np.empty(n, dtype=np.float32)
    lib().oracle_rand_sequence(px, py, f, n, _fp(out))
    return out


BUILTINS = {"sin": 0, "cos": 1, "log": 2, "acos": 3, "atan2": 4, "fract": 5, "sqrt": 6, "inversesqrt": 7}


def eval_builtin(name, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    yy = None if y is None else np.ascontiguousarray(y, dtype=np.float32)
    lib().oracle_eval_builtin(BUILTINS[name], _fp(x), None if yy is None else _fp(yy), _fp(out), x.size)
    return out
