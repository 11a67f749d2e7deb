"""CPU tests of the drop-in boundary (include/rt/*.h) — no compute calls, no GPU needed.

* every function the headers declare is exported by the in-tree libraries;
* the host-only entry points (stripe arithmetic, de-interleave, frame random
  factors, the threaded-BVH re-layout) agree with independent restatements;
* failures are reported with codes and messages, never silently.
"""
import ctypes
import os
import re
import subprocess
import zlib

import numpy as np
import pytest

import rtamd
from rtamd import _lib
from rtamd import scene as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(REPO, "include", "rt")


def declared(header):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(rts?_\w+)\s*\(", src, flags=re.M)))


def exported(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(_lib.LIB_DIR, lib)], text=True)
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


@pytest.mark.parametrize("header,lib", [("rt.h", "librtamd.so"), ("rt_debug.h", "librtamd.so"),
                                        ("rt_scene.h", "librtscene.so")])
def test_header_symbols_exported(header, lib):
    names = declared(header)
    assert len(names) >= 5, names
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, f"{lib} lacks {missing}"


def test_rt_h_declares_the_boundary():
    names = set(declared("rt.h"))
    for n in ["rt_create", "rt_destroy", "rt_last_error", "rt_upload_buffer", "rt_upload_texture", "rt_set_camera",
              "rt_set_params", "rt_resize", "rt_render", "rt_sync", "rt_read_image", "rt_write_image",
              "rt_set_partition", "rt_bind_device_image", "rt_set_stream"]:
        assert n in names, n


def test_abi_version():
    assert rtamd.amd().rt_abi_version() == 1


@pytest.mark.skipif(rtamd.amd().rt_debug_device_count() > 0, reason="a HIP device is visible")
def test_create_without_device_fails_loudly():
    L = rtamd.amd()
    h = ctypes.c_void_p()
    rc = L.rt_create(1, None, ctypes.byref(h))
    assert rc == -2 and not h.value                   # RT_ERR_DEVICE
    assert b"no HIP device" in L.rt_last_error(None)
    with pytest.raises(rtamd.RTError, match="no HIP device"):
        rtamd.RenderContext()


def test_null_context_calls_are_rejected():
    L = rtamd.amd()
    assert L.rt_render(None, 1, 1, None) == -1
    assert L.rt_resize(None, 8, 8) == -1
    assert L.rt_destroy(None) == -1


@pytest.mark.parametrize("seed", [0, 1, 12345, 2 ** 63 + 5])
def test_frame_rand_factor(seed):
    L = rtamd.amd()
    py = rtamd.frame_rand_factors(seed, 0, 300)
    c = np.array([L.rt_frame_rand_factor(ctypes.c_uint64(seed), ctypes.c_uint64(f)) for f in range(300)], np.float32)
    assert np.array_equal(py, c)
    assert np.all(py >= 0) and np.all(py < 1)
    assert np.array_equal(rtamd.frame_rand_factors(seed, 100, 50), py[100:150])


def test_stripe_arithmetic():
    L = rtamd.amd()
    for H in [1, 7, 16, 37, 1080]:
        for world in [1, 2, 3, 8]:
            for stripe in [1, 4, 16, 64]:
                total = 0
                padded = rtamd.padded_local_rows(H, world, stripe)
                assert L.rt_padded_local_rows(H, world, stripe) == padded
                owned = []
                for r in range(world):
                    n = rtamd.local_rows(H, r, world, stripe)
                    assert L.rt_local_rows(H, r, world, stripe) == n <= padded
                    rows = rtamd.stripe_rows_of(H, r, world, stripe)
                    assert len(rows) == n and all((y // stripe) % world == r for y in rows)
                    owned += list(rows)
                    total += n
                assert total == H and sorted(owned) == list(range(H))


@pytest.mark.parametrize("H,W,world,stripe", [(37, 5, 3, 4), (1080, 3, 8, 16), (9, 2, 2, 16), (2160, 2, 8, 8),
                                              (45, 4, 5, 64), (7, 3, 8, 1)])
def test_deinterleave_matches(H, W, world, stripe):
    L = rtamd.amd()
    padded = rtamd.padded_local_rows(H, world, stripe)
    g = np.random.default_rng(1).random((world, padded, W, 4), dtype=np.float32)
    out = np.zeros((H, W, 4), np.float32)
    fp = lambda a: a.ctypes.data_as(_lib.c_float_p)  # noqa: E731
    assert L.rt_deinterleave_rows(fp(g), W, H, world, stripe, fp(out)) == 0
    assert np.array_equal(out, rtamd.deinterleave(g, H, world, stripe))
    # the device gather's indexing (deinterleave_kernel / rt_gathered_row), run on the host
    dev = np.zeros((H, W, 4), np.float32)
    assert L.rt_debug_deinterleave(fp(g), W, H, world, stripe, fp(dev)) == 0
    assert np.array_equal(dev, out)


# --- threaded BVH == the reference's stack traversal order --------------------------------------

DNODE = np.dtype([("box", "<f4", 6), ("meta", "<u4"), ("prims", "<u4")])


def threaded(nodes_bytes):
    L = rtamd.amd()
    n = ctypes.c_int()
    assert L.rt_debug_threaded_bvh(nodes_bytes, len(nodes_bytes), None, 0, ctypes.byref(n)) == 0
    out = ctypes.create_string_buffer(n.value * 32)
    assert L.rt_debug_threaded_bvh(nodes_bytes, len(nodes_bytes), out, len(out), ctypes.byref(n)) == 0
    return np.frombuffer(out.raw, dtype=DNODE)


def _pred(box, seed, p):
    return zlib.crc32(box.tobytes() + seed.to_bytes(4, "little")) % 1000 < p


def stack_visits(nodes_bytes, seed, p):
    """compute.glsl:225-263: pop, test AABB, leaf -> test left/right models, inner -> push left then right."""
    raw = np.frombuffer(nodes_bytes, dtype=np.uint8).reshape(-1, 32)
    box = raw[:, :24].copy().view(np.float32).reshape(-1, 6)
    ids = raw[:, 24:].copy().view(np.int32).reshape(-1, 2)
    seq, stack = [], [0]
    while stack:
        k = stack.pop()
        hit = _pred(box[k], seed, p)
        lt = ids[k, 0] & 0xFFFF
        rt = ids[k, 1] & 0xFFFF
        if lt and ids[k, 0] == ids[k, 1] and lt != 3:
            rt = 0   # re-layout drops the redundant second test of a non-medium singleton leaf
        leaf = (lt, (ids[k, 0] >> 16) & 0xFFFF, rt, (ids[k, 1] >> 16) & 0xFFFF) if lt else None
        seq.append((box[k].tobytes(), hit, leaf if hit else None))
        if hit and not lt:
            stack += [(ids[k, 0] >> 16) & 0xFFFF, (ids[k, 1] >> 16) & 0xFFFF]
    return seq


def threaded_visits(dn, seed, p):
    """The kernel's walk: hit inner -> next record; leaf or miss -> skip link (0xFFFF = end)."""
    seq, i = [], 0
    while i != 0xFFFF:
        m = int(dn[i]["meta"])
        lt, rt = (m >> 16) & 0xF, (m >> 20) & 0xF
        hit = _pred(dn[i]["box"], seed, p)
        pr = int(dn[i]["prims"])
        seq.append((dn[i]["box"].tobytes(), hit, (lt, pr & 0xFFFF, rt, pr >> 16) if (hit and lt) else None))
        i = i + 1 if (hit and not lt) else m & 0xFFFF
    return seq


@pytest.mark.parametrize("sid", [0, 6, 8])
def test_threaded_bvh_visit_order(sid):
    sc = rtamd.Scene(sid, 32, 32, seed=1)
    nb = sc.buffers[S.BIND_BVH]
    dn = threaded(nb)
    assert len(dn) == sc.info["n_bvh_nodes"]
    for seed in range(12):
        for p in (1000, 700, 300):
            assert threaded_visits(dn, seed, p) == stack_visits(nb, seed, p), (seed, p)


def test_threaded_bvh_rejects_bad_trees():
    L = rtamd.amd()
    n = ctypes.c_int()
    # inner node whose child index is out of range
    bad = np.zeros(1, dtype=[("box", "<f4", 6), ("l", "<i4"), ("r", "<i4")])
    bad["l"], bad["r"] = 5 << 16, 6 << 16
    assert L.rt_debug_threaded_bvh(bad.tobytes(), 32, None, 0, ctypes.byref(n)) == -1
    # a self-referencing chain deeper than the reference's stack[64]
    deep = np.zeros(1, dtype=bad.dtype)
    deep["l"], deep["r"] = 0, 0
    assert L.rt_debug_threaded_bvh(deep.tobytes(), 32, None, 0, ctypes.byref(n)) != 0
    # size not a multiple of the 32-byte record
    assert L.rt_debug_threaded_bvh(b"\0" * 33, 33, None, 0, ctypes.byref(n)) == -1
