"""Render context and the RaytraceExecutor mirror over the rt.h C ABI.

``RenderContext`` owns an ``rt_ctx`` (one or more MI355X devices, or one
stripe-partition of a multi-process render) and uploads a ``Scene`` the way the
reference's Java side fills its SSBOs/UBO/textures.  ``RaytraceExecutor``
restates J/system/RaytraceExecutor.java (setSamplePerPixel, raytrace,
sampleComplete, resetCompleteState, completion listeners) with frames batched
per kernel launch instead of one dispatch per vsync.
"""
import ctypes
import time

import numpy as np

from . import _lib
from ._lib import RTError, c_float_p
from .scene import Scene, spp_uniforms

MASK64 = (1 << 64) - 1


def frame_rand_factors(seed, start, n):
    """u_rand_factor for frames [start, start+n): top 24 bits of
    splitmix64(seed, frame)/2^24 (rt.h rt_frame_rand_factor; stands in for the
    reference's per-frame (float)Math.random(), RaytraceExecutor.java:124)."""
    out = np.empty(n, dtype=np.float32)
    for k in range(n):
        z = (seed + (start + k + 1) * 0x9E3779B97F4A7C15) & MASK64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        z ^= z >> 31
        out[k] = np.float32(z >> 40) / np.float32(16777216.0)
    return out


def comm_unique_id(lib=None):
    """rt_comm_unique_id: a fresh 128-byte RCCL communicator id (rank 0 makes it, the host
    hands it to every rank)."""
    L = lib or _lib.amd()
    buf = ctypes.create_string_buffer(128)
    rc = L.rt_comm_unique_id(buf)
    if rc != 0:
        raise RTError(rc, "rt_comm_unique_id failed (RCCL unavailable)")
    return buf.raw


def sah_bvh(scene, order=2, eye=None, prim_cost=1.0, lib=None):
    """rt_debug_build_sah_bvh (no device needed): the RT_BVH_SAH tree of a Scene's prims, as the
    reference's BVH bytes (binding 1).  order 2 with the camera position (the default) is
    rt_set_bvh_mode's tree."""
    L = lib or _lib.amd()
    b = scene.buffers
    keep = [ctypes.create_string_buffer(b[k], len(b[k])) if b[k] else None for k in range(6)]
    e = (ctypes.c_float * 3)(*(eye if eye is not None else scene.camera[4:7]))
    n = ctypes.c_size_t()
    args = (keep[0], len(b[0]), keep[2], len(b[2]), keep[3], len(b[3]), keep[4], len(b[4]), keep[1], len(b[1]),
            int(order), e, float(prim_cost))
    rc = L.rt_debug_build_sah_bvh(*args, None, 0, ctypes.byref(n))
    if rc != 0:
        raise RTError(rc, "rt_debug_build_sah_bvh failed")
    out = ctypes.create_string_buffer(max(1, n.value))
    rc = L.rt_debug_build_sah_bvh(*args, out, n.value, ctypes.byref(n))
    if rc != 0:
        raise RTError(rc, "rt_debug_build_sah_bvh failed")
    return out.raw[:n.value]


def local_rows(height, rank, world, stripe_rows):
    n_stripes = (height + stripe_rows - 1) // stripe_rows
    return sum(min(stripe_rows, height - s * stripe_rows) for s in range(rank, n_stripes, world))


def padded_local_rows(height, world, stripe_rows):
    n_stripes = (height + stripe_rows - 1) // stripe_rows
    return ((n_stripes + world - 1) // world) * stripe_rows


def stripe_rows_of(height, rank, world, stripe_rows):
    """Global row indices owned by `rank`, in local (compact) order."""
    n_stripes = (height + stripe_rows - 1) // stripe_rows
    rows = []
    for s in range(rank, n_stripes, world):
        rows.extend(range(s * stripe_rows, min(height, (s + 1) * stripe_rows)))
    return np.array(rows, dtype=np.int64)


def deinterleave(gathered, height, world, stripe_rows):
    """[world, padded_rows, W, 4] gathered stripe blocks -> [H, W, 4] image."""
    W = gathered.shape[2]
    out = np.zeros((height, W, 4), dtype=gathered.dtype)
    for k in range(world):
        rows = stripe_rows_of(height, k, world, stripe_rows)
        out[rows] = gathered[k, :len(rows)]
    return out


# rt_debug.h RT_OPTION_*: per-context options set by explicit calls (the release library
# reads no environment).  Below 100 they never change a bit of the image; 100+ exist in
# the A/B build only.
OPTIONS = {"box_pretest": 1, "fastdiv": 2, "sph_lds": 3, "big_wg": 4, "chunk_target": 5,
           "staged_chunk_target": 6, "stage_tiles": 7, "sm_batch": 8, "sm_frac": 9, "walk_frac": 10,
           "watchdog_ms": 11, "chunk_wait_ms": 12, "lds_node_cap": 13, "compact_boxes": 14, "spine": 15,
           "tl_leaf_lds": 16, "perlin_packed": 17, "sparse_stage": 18, "sphere_pairs": 19, "leaf_prefetch": 20, "tl_small_lds": 21, "shade_lds": 22, "box_vnodes": 23, "zero_dir_end": 24, "collapse": 25, "rebuild": 26, "tail_chunks": 27, "kernel_variant": 100, "debug_flags": 101}
# rt_debug_last_launch fields
LAUNCH_FIELDS = ("shape", "block", "fastdiv", "pretest", "lds_bytes", "lds_nodes", "box_records", "staged",
                 "chunks", "spine", "sparse", "sphere_pairs", "leaf_prefetch", "shade_lds", "walk_frac", "bvh_mode",
                 "box_vnodes", "collapsed", "rebuilt")
BVH_MODES = {"reference": 0, "sah": 1}   # rt.h RT_BVH_*
SHAPES = {0: "fast-lds", 1: "fast-global", 2: "link-lds", 3: "meta-lds", 4: "meta-global", 5: "link-two-level"}


class RenderContext:
    """An rt_ctx: device buffers, accumulation image and launch state.

    ``options`` (dict name -> int, see OPTIONS) are applied right after creation;
    ``ab=True`` uses the A/B build (librtamd_ab.so) for kernel-variant options; ``lib`` a
    library at that path (tools/lib_ab.py)."""

    def __init__(self, devices=(0,), rank=0, world=1, stripe_rows=16, options=None, ab=False, lib=None):
        L = _lib.amd_at(lib) if lib else (_lib.amd_ab() if ab else _lib.amd())
        self._L = L
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        rc = L.rt_create(len(devices), devs, ctypes.byref(h))
        if rc != 0:
            raise RTError(rc, L.rt_last_error(None).decode())
        self._h = h
        self.devices = tuple(devices)
        self.rank, self.world, self.stripe_rows = rank, world, stripe_rows
        if world > 1 or stripe_rows != 16:
            self._check(L.rt_set_partition(h, rank, world, stripe_rows))
        self.width = self.height = 0
        self.max_depth = 5
        self.background = np.zeros(3, np.float32)
        self.sqrt_spp, self.recip_sqrt_spp = 1.0, 1.0
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_bvh_mode(self, mode):
        """rt_set_bvh_mode: "reference" (default, bit-exact) or "sah" (non-parity fast mode)."""
        self._check(self._L.rt_set_bvh_mode(self._h, BVH_MODES[mode] if isinstance(mode, str) else int(mode)))

    def walk_bvh(self):
        """rt_debug_walk_bvh: the BVH bytes (reference node format) the link walk runs on."""
        n = ctypes.c_size_t()
        self._check(self._L.rt_debug_walk_bvh(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(1, n.value))
        self._check(self._L.rt_debug_walk_bvh(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def set_option(self, name, value):
        """rt_debug_set_option (rt_debug.h RT_OPTION_*)."""
        self._check(self._L.rt_debug_set_option(self._h, OPTIONS[name], int(value)))

    def get_option(self, name):
        v = ctypes.c_int()
        self._check(self._L.rt_debug_get_option(self._h, OPTIONS[name], ctypes.byref(v)))
        return v.value

    def count_node_hits(self, on=True):
        """rt_debug_count_node_hits: arm (and zero) the stats twin's per-node hit count."""
        self._check(self._L.rt_debug_count_node_hits(self._h, 1 if on else 0))

    def read_node_hits(self):
        """rt_debug_read_node_hits -> (hits per link node as uint32 array, walks begun at the root)."""
        n = ctypes.c_size_t()
        self._check(self._L.rt_debug_read_node_hits(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, np.uint32)
        self._check(self._L.rt_debug_read_node_hits(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)),
                                                     out.size, ctypes.byref(n)))
        return out[:-1].copy(), int(out[-1])

    def set_collapse_hits(self, hits, walks):
        """rt_debug_set_collapse_hits: plan the collapse from measured hits (empty: the camera grid)."""
        h = np.ascontiguousarray(hits, np.uint32)
        self._check(self._L.rt_debug_set_collapse_hits(self._h, h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)),
                                                        h.size, int(walks)))

    def last_launch(self):
        """rt_debug_last_launch as a dict (the launch shape the last rt_render took)."""
        out = (ctypes.c_int * 20)()
        self._check(self._L.rt_debug_last_launch(self._h, out, 20))
        d = dict(zip(LAUNCH_FIELDS, out[:len(LAUNCH_FIELDS)]))
        d["shape_name"] = SHAPES.get(d["shape"], "?")
        return d

    def _check(self, rc):
        if rc != 0:
            raise RTError(rc, self._L.rt_last_error(self._h).decode())
        return rc

    # -- scene upload (RaytraceModel.putModelsToProgram, Texture.putData, Camera.init)
    def upload_scene(self, scene: Scene):
        for b in range(6):
            data = scene.buffers[b]
            buf = ctypes.create_string_buffer(data, len(data)) if data else None
            self._check(self._L.rt_upload_buffer(self._h, b, buf, len(data)))
        for t in scene.textures:
            buf = ctypes.create_string_buffer(t.data, len(t.data))
            self._check(self._L.rt_upload_texture(self._h, t.slot, t.format, t.width, t.height, buf))
        self.set_camera(scene.camera)
        self.background = scene.background.copy()

    def set_camera(self, ubo):
        ubo = np.ascontiguousarray(ubo, dtype=np.float32)
        assert ubo.size == 28
        self._check(self._L.rt_set_camera(self._h, ubo.ctypes.data_as(c_float_p)))

    def set_params(self, max_depth=None, background=None, spp=None, uniforms=None):
        """uniforms = (sqrt_spp, recip_sqrt_spp) as raw floats, instead of spp's."""
        if max_depth is not None:
            self.max_depth = int(max_depth)
        if background is not None:
            self.background = np.asarray(background, np.float32)
        if spp is not None:
            self.sqrt_spp, self.recip_sqrt_spp = spp_uniforms(spp)
        if uniforms is not None:
            self.sqrt_spp, self.recip_sqrt_spp = float(np.float32(uniforms[0])), float(np.float32(uniforms[1]))
        bg = np.ascontiguousarray(self.background, dtype=np.float32)
        self._check(self._L.rt_set_params(self._h, self.max_depth, bg.ctypes.data_as(c_float_p),
                                          self.sqrt_spp, self.recip_sqrt_spp))

    def resize(self, width, height):
        self._check(self._L.rt_resize(self._h, int(width), int(height)))
        self.width, self.height = int(width), int(height)

    @property
    def local_rows(self):
        if len(self.devices) > 1:
            return self.height
        return local_rows(self.height, self.rank, self.world, self.stripe_rows)

    @property
    def padded_rows(self):
        return padded_local_rows(self.height, self.world, self.stripe_rows)

    def render(self, first_frame, rand_factors):
        rf = np.ascontiguousarray(rand_factors, dtype=np.float32)
        self._check(self._L.rt_render(self._h, int(first_frame), int(rf.size), rf.ctypes.data_as(c_float_p)))

    def sync(self):
        self._check(self._L.rt_sync(self._h))

    def last_render_ns(self):
        v = ctypes.c_uint64()
        self._check(self._L.rt_last_render_ns(self._h, ctypes.byref(v)))
        return v.value

    def render_done(self):
        """rt_render_done: the last render's device ns once it finished, else None (no wait)."""
        v = ctypes.c_uint64()
        rc = self._L.rt_render_done(self._h, ctypes.byref(v))
        if rc < 0:
            self._check(rc)
        return v.value if rc == 1 else None

    def read_image(self):
        """[local_rows, W, 4] float32 (the full image for an unpartitioned context)."""
        out = np.empty((self.local_rows, self.width, 4), dtype=np.float32)
        self._check(self._L.rt_read_image(self._h, out.ctypes.data_as(c_float_p)))
        return out

    def write_image(self, rgba):
        rgba = np.ascontiguousarray(rgba, dtype=np.float32)
        self._check(self._L.rt_write_image(self._h, rgba.ctypes.data_as(c_float_p)))

    # -- RCCL behind the ABI (rt.h rt_comm_*): one process per GPU
    def comm_init(self, uid, rank, world):
        """rt_comm_init with the 128-byte id rank 0 made (comm_unique_id)."""
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        self._check(self._L.rt_comm_init(self._h, buf, int(rank), int(world)))

    def comm_set_timeout(self, timeout_ms):
        """rt_comm_set_timeout: deadline of comm_init / gather_image in ms (0 = none); past it the
        call raises RTError(RT_ERR_TIMEOUT) with the communicator aborted."""
        self._check(self._L.rt_comm_set_timeout(self._h, int(timeout_ms)))

    def comm_abort(self):
        """rt_comm_abort: abort the communicator and free its queued work."""
        self._check(self._L.rt_comm_abort(self._h))

    def gather_image(self):
        """rt_gather_image: the full [H, W, 4] image on rank 0 (None on the other ranks)."""
        if self.rank == 0:
            out = np.empty((self.height, self.width, 4), dtype=np.float32)
            self._check(self._L.rt_gather_image(self._h, out.ctypes.data_as(c_float_p)))
            return out
        self._check(self._L.rt_gather_image(self._h, None))
        return None

    def gather_path(self):
        """How the last gather ran: 'host', 'peer' (device copies) or 'rccl' (None before any)."""
        return {0: "host", 1: "peer", 2: "rccl"}.get(self._L.rt_gather_path(self._h))

    def bind_device_image(self, ptr, nbytes):
        self._check(self._L.rt_bind_device_image(self._h, ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes)))

    def set_stream(self, stream_ptr):
        self._check(self._L.rt_set_stream(self._h, ctypes.c_void_p(stream_ptr)))

    def close(self):
        if getattr(self, "_h", None):
            self._L.rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RaytraceExecutor:
    """J/system/RaytraceExecutor.java over an rt_ctx.

    One reference ``raytrace()`` = one dispatch = one frame (1 spp) per vsync;
    here ``raytrace(n)`` queues n frames in one rt_render call, with the same
    per-frame uniforms (frame_count = ++numSamples, u_rand_factor).
    """

    def __init__(self, ctx: RenderContext, seed=1):
        self.ctx = ctx
        self.seed = seed
        self._listeners = []
        self.samplePerPixel = 0
        self.resetCompleteState()
        self.lastDispatchTime = 0

    def setSamplePerPixel(self, spp):            # :50-56
        self.samplePerPixel = int(spp)
        self.ctx.set_params(spp=spp)

    def resetCompleteState(self):                # :58-62
        self.isSampleComplete = False
        self.numSamples = 0
        self.finishTime = -1

    def getNumSamples(self):
        return self.numSamples

    def getSamplePerPixel(self):
        return self.samplePerPixel

    def getFinishTime(self):
        return self.finishTime

    def getFinishTimeString(self):               # :76-89
        ms = self.finishTime
        hours, minutes, seconds = ms // 3600000, (ms // 60000) % 60, (ms // 1000) % 60
        s = (f"{hours}hour " if hours > 0 else "") + (f"{minutes}minutes " if minutes > 0 else "")
        return s + f"{seconds}.{ms % 1000}seconds"

    def getLastDispatchTime(self):
        return self.lastDispatchTime

    def addCompleteListener(self, fn):           # :96-98
        self._listeners.append(fn)

    def raytrace(self, n_frames=1):              # :100-142
        if self.numSamples == 0:
            self._start = time.time()
        # the previous call's device time once it is available, without waiting (:106-115)
        done = self.ctx.render_done() if self.numSamples else None
        if done is not None:
            self.lastDispatchTime = done // 1_000_000
        n = max(0, min(int(n_frames), self.samplePerPixel - self.numSamples)) if self.samplePerPixel else int(n_frames)
        if n == 0:
            return
        rf = frame_rand_factors(self.seed, self.numSamples, n)
        self.ctx.render(self.numSamples + 1, rf)
        self.numSamples += n

    def sampleComplete(self):                    # :144-156
        if not self.isSampleComplete:
            self.isSampleComplete = self.numSamples >= self.samplePerPixel
            if self.isSampleComplete:
                self.ctx.sync()
                self.lastDispatchTime = self.ctx.last_render_ns() // 1_000_000
                self.finishTime = int((time.time() - self._start) * 1000)
                for fn in self._listeners:
                    fn()
        return self.isSampleComplete
