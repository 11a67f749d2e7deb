"""ctypes loaders for the in-tree native libraries.

* ``librtamd.so``    — the HIP kernel behind the C ABI of include/rt/rt.h (release:
  one kernel structure, no environment knobs).
* ``librtamd_ab.so`` — the same ABI built with -DRT_AB_KNOBS: the A/B kernel
  structures, stats kernels and RT_* environment knobs (variant tests, tools/).
* ``librtscene.so``  — the host scene builder of include/rt/rt_scene.h.

All are built in-tree by ``make -C raytracing-book_amd`` (see
__graft_entry__.build()).  There is no Python or CPU fallback for the render
path: if the library is missing, loading raises.  ``amd()`` is the release
library unless the harness sets RTAMD_LIB=ab (tools/ab_variants.py).
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
ASSET_DIR = os.path.join(REPO_DIR, "assets")

c_float_p = ctypes.POINTER(ctypes.c_float)
c_int_p = ctypes.POINTER(ctypes.c_int)

_amd = None
_amd_ab = None
_scene = None


class RTError(RuntimeError):
    """A negative status from the C ABI, with rt_last_error()'s message."""

    def __init__(self, code, msg):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


def _load(name):
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `make -C {PKG_DIR}` "
            "(or __graft_entry__.build()); there is no fallback path")
    return ctypes.CDLL(path)


def _proto(lib, name, restype, *argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = list(argtypes)
    return fn


class RtsInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "scene_id", "width", "height", "n_spheres", "n_quads", "n_boxes", "n_media",
        "n_lights", "n_bvh_nodes", "n_bvh_prims", "bvh_depth", "max_stack", "n_textures")] + [
        ("background", ctypes.c_float * 3)]


class RtsCamera(ctypes.Structure):
    _fields_ = [("look_from", ctypes.c_float * 3), ("look_at", ctypes.c_float * 3), ("vup", ctypes.c_float * 3),
                ("vfov", ctypes.c_float), ("defocus_angle", ctypes.c_float), ("focus_dist", ctypes.c_float),
                ("background", ctypes.c_float * 3)]


def _amd_protos(L):
    vp, sz, i, f, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_float, ctypes.c_uint64
    _proto(L, "rt_abi_version", i)
    _proto(L, "rt_create", i, i, c_int_p, ctypes.POINTER(vp))
    _proto(L, "rt_destroy", i, vp)
    _proto(L, "rt_last_error", ctypes.c_char_p, vp)
    _proto(L, "rt_upload_buffer", i, vp, i, vp, sz)
    _proto(L, "rt_upload_texture", i, vp, i, i, i, i, vp)
    _proto(L, "rt_set_camera", i, vp, c_float_p)
    _proto(L, "rt_set_params", i, vp, i, c_float_p, f, f)
    _proto(L, "rt_resize", i, vp, i, i)
    _proto(L, "rt_render", i, vp, i, i, c_float_p)
    _proto(L, "rt_sync", i, vp)
    _proto(L, "rt_read_image", i, vp, c_float_p)
    _proto(L, "rt_write_image", i, vp, c_float_p)
    _proto(L, "rt_last_render_ns", i, vp, ctypes.POINTER(u64))
    _proto(L, "rt_render_done", i, vp, ctypes.POINTER(u64))
    _proto(L, "rt_set_partition", i, vp, i, i, i)
    _proto(L, "rt_local_rows", i, i, i, i, i)
    _proto(L, "rt_padded_local_rows", i, i, i, i)
    _proto(L, "rt_bind_device_image", i, vp, vp, sz)
    _proto(L, "rt_set_stream", i, vp, vp)
    _proto(L, "rt_deinterleave_rows", i, c_float_p, i, i, i, i, c_float_p)
    _proto(L, "rt_frame_rand_factor", f, u64, u64)
    _proto(L, "rt_comm_unique_id", i, vp)
    _proto(L, "rt_comm_init", i, vp, vp, i, i)
    _proto(L, "rt_gather_image", i, vp, c_float_p)
    _proto(L, "rt_gather_path", i, vp)
    _proto(L, "rt_comm_set_timeout", i, vp, i)
    _proto(L, "rt_comm_abort", i, vp)
    _proto(L, "rt_debug_eval_builtin", i, i, i, c_float_p, c_float_p, c_float_p, i)
    _proto(L, "rt_debug_threaded_bvh", i, vp, sz, vp, sz, c_int_p)
    _proto(L, "rt_debug_fast_tables", i, vp, sz, vp, sz, vp, sz, i, vp, sz, c_int_p,
           ctypes.POINTER(ctypes.c_uint32), sz, c_int_p, c_int_p)
    _proto(L, "rt_debug_link_nodes", i, vp, sz, vp, sz, c_int_p)
    _proto(L, "rt_debug_collapse_links", i, vp, sz, vp, i, i, i, vp, sz, c_int_p, vp, sz, c_int_p)
    _proto(L, "rt_debug_link_nodes_vbox", i, vp, sz, c_float_p, i, vp, sz, c_int_p, c_int_p)
    _proto(L, "rt_debug_box_records", i, vp, sz, vp, sz, c_int_p)
    _proto(L, "rt_debug_perlin_pack", i, c_float_p, i, i, vp, sz)
    _proto(L, "rt_debug_sphere_pair_leaves", i, vp, sz, c_int_p)
    _proto(L, "rt_debug_deinterleave", i, c_float_p, i, i, i, i, c_float_p)
    _proto(L, "rt_debug_device_count", i)
    _proto(L, "rt_debug_enable_stats", i, vp, i)
    _proto(L, "rt_debug_read_stats", i, vp, ctypes.POINTER(ctypes.c_ulonglong), i)
    _proto(L, "rt_debug_read_census", i, vp, ctypes.POINTER(ctypes.c_uint), ctypes.c_size_t,
           ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
    _proto(L, "rt_debug_count_node_hits", i, vp, i)
    _proto(L, "rt_debug_read_node_hits", i, vp, ctypes.POINTER(ctypes.c_uint), ctypes.c_size_t,
           ctypes.POINTER(ctypes.c_size_t))
    _proto(L, "rt_debug_set_collapse_hits", i, vp, ctypes.POINTER(ctypes.c_uint), ctypes.c_size_t,
           ctypes.c_ulonglong)
    _proto(L, "rt_debug_ab_build", i)
    _proto(L, "rt_debug_set_option", i, vp, i, i)
    _proto(L, "rt_debug_get_option", i, vp, i, c_int_p)
    _proto(L, "rt_debug_last_launch", i, vp, c_int_p, i)
    _proto(L, "rt_set_bvh_mode", i, vp, i)
    _proto(L, "rt_debug_walk_bvh", i, vp, vp, sz, ctypes.POINTER(sz))
    _proto(L, "rt_debug_build_sah_bvh", i, vp, sz, vp, sz, vp, sz, vp, sz, vp, sz, i, c_float_p, f, vp, sz,
           ctypes.POINTER(sz))
    return L


def _import_torch_first():
    # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7, the name librtamd needs): loaded first, it is the one
    # librtamd binds to, so torch tensors/streams handed to rt_bind_device_image /
    # rt_set_stream belong to the same runtime.  Loaded after /opt/rocm's copy,
    # torch would bring a second runtime that sees no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def amd():
    """The product library (HIP), or the A/B build when RTAMD_LIB=ab.  Raises
    ImportError when it was not built."""
    global _amd
    if os.environ.get("RTAMD_LIB") == "ab":
        return amd_ab()
    if _amd is None:
        _import_torch_first()
        _amd = _amd_protos(_load("librtamd.so"))
    return _amd


def amd_ab():
    """The A/B build of the same ABI (kernel variants, stats kernels, RT_* knobs)."""
    global _amd_ab
    if _amd_ab is None:
        _import_torch_first()
        _amd_ab = _amd_protos(_load("librtamd_ab.so"))
    return _amd_ab


_amd_at = {}


def amd_at(path):
    """Another build of the same ABI loaded from `path` (tools/lib_ab.py: a previous
    revision's kernel timed beside the current one in one process)."""
    path = os.path.abspath(path)
    if path not in _amd_at:
        if not os.path.exists(path):
            raise ImportError(f"{path} is missing")
        _import_torch_first()
        _amd_at[path] = _amd_protos(ctypes.CDLL(path))
    return _amd_at[path]


def scene_lib():
    """The host scene builder (no GPU needed)."""
    global _scene
    if _scene is None:
        L = _load("librtscene.so")
        vp, sz, i, f = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_float
        _proto(L, "rts_build", i, i, i, i, ctypes.c_uint64, ctypes.c_char_p, ctypes.POINTER(vp))
        _proto(L, "rts_free", None, vp)
        _proto(L, "rts_last_error", ctypes.c_char_p)
        _proto(L, "rts_decode_image", i, ctypes.c_char_p, c_int_p, c_int_p, c_int_p,
               ctypes.POINTER(ctypes.c_uint8), sz)
        _proto(L, "rts_decode_last_error", ctypes.c_char_p)
        _proto(L, "rts_get_info", i, vp, ctypes.POINTER(RtsInfo))
        _proto(L, "rts_get_buffer", i, vp, i, ctypes.POINTER(vp), ctypes.POINTER(sz))
        _proto(L, "rts_get_texture", i, vp, i, c_int_p, c_int_p, c_int_p, ctypes.POINTER(vp), ctypes.POINTER(sz))
        _proto(L, "rts_get_camera", i, vp, c_float_p)
        _proto(L, "rts_set_image_size", i, vp, i, i)
        _proto(L, "rts_spp_uniforms", None, i, c_float_p, c_float_p)
        _proto(L, "rts_tonemap_rgb8", i, c_float_p, i, i, ctypes.POINTER(ctypes.c_uint8))
        _proto(L, "rts_save_png", i, c_float_p, i, i, ctypes.c_char_p)
        _proto(L, "rts_java_random_next_int", ctypes.c_int32, ctypes.c_int64, i)
        _proto(L, "rts_java_random_next_double", ctypes.c_double, ctypes.c_int64, i)
        _proto(L, "rts_java_random_next_float", f, ctypes.c_int64, i)
        _proto(L, "rts_java_random_next_int_bound", ctypes.c_int32, ctypes.c_int64, i)
        f3 = ctypes.POINTER(ctypes.c_float)
        _proto(L, "rts_new", i, ctypes.c_uint64, ctypes.c_char_p, ctypes.POINTER(vp))
        _proto(L, "rts_solid_texture", i, vp, f, f, f, c_int_p)
        _proto(L, "rts_checker_texture", i, vp, f3, f3, f, c_int_p)
        _proto(L, "rts_perlin_texture", i, vp, f, c_int_p)
        _proto(L, "rts_image_texture", i, vp, ctypes.c_char_p, i, i, c_int_p)
        _proto(L, "rts_material", i, vp, i, i, f, f3, c_int_p)
        _proto(L, "rts_sphere", i, vp, f3, f3, f, i, c_int_p)
        _proto(L, "rts_quad", i, vp, f3, f3, f3, i, c_int_p)
        _proto(L, "rts_box", i, vp, f3, f3, f3, f3, i, c_int_p)
        _proto(L, "rts_constant_medium", i, vp, i, f, i, c_int_p)
        _proto(L, "rts_add_model", i, vp, i)
        _proto(L, "rts_add_light", i, vp, i)
        _proto(L, "rts_camera", i, vp, ctypes.POINTER(RtsCamera))
        _proto(L, "rts_finish", i, vp, i, i)
        _scene = L
    return _scene
