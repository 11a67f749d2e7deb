"""The link-format BVH the default kernel walks (rt_capi.hip build_links,
rt_device.h RT_LINK_*; rt_kernel.hip trace with WHILE_WHILE bit 8) — host-side,
no GPU needed.

Every node keeps the threaded node's box; its hit / miss words are the
threaded walk's successors as byte offsets, and a hit leaf leaves the loop
with its leaf ordinal.  Under any pattern of box hits the link walk visits the
same nodes and tests the same leaves, in the same order, as the threaded walk
(which itself replays the reference's stack walk, test_abi.py).
"""
import ctypes

import numpy as np
import pytest

import rtamd
from test_fast_tables import END, is_leaf, threaded

LEAF, LEND = 0x80000000, 0xFFFFFFFF


def links(scene):
    L = rtamd.amd()
    b = scene.buffers[1]
    bvh = ctypes.create_string_buffer(b, len(b))
    n = ctypes.c_int()
    assert L.rt_debug_link_nodes(bvh, len(b), None, 0, ctypes.byref(n)) == 0
    out = np.zeros((max(n.value, 1), 4), np.float32)
    assert L.rt_debug_link_nodes(bvh, len(b), out.ctypes.data, out.nbytes, ctypes.byref(n)) == 0
    return out[:n.value]


def walk_threaded(tn, hits):
    i, seen, tested = 0, [], []
    while i != END:
        seen.append(i)
        nd = tn[i]
        skip = int(nd["meta"]) & 0xFFFF
        if not hits[i]:
            i = skip
        elif is_leaf(nd):
            tested.append((int(nd["meta"]) & 0xFF0000, int(nd["prims"])))
            i = skip
        else:
            i += 1
    return seen, tested


def walk_links(ln, n, hits):
    words = ln.view(np.uint32)
    leaves = words[2 * n:].reshape(-1, 2)
    nx, seen, tested = 0, [], []
    while True:
        while nx < LEAF:
            k = nx // 32
            seen.append(k)
            nx = int(words[2 * k + 1, 2] if hits[k] else words[2 * k + 1, 3])
        if nx == LEND:
            break
        lf = leaves[(nx >> 16) & 0x7FFF]
        tested.append((int(lf[0]), int(lf[1])))
        nx &= 0xFFFF
        if nx == 0xFFFF:
            break
    return seen, tested


@pytest.mark.parametrize("sid", range(10))
def test_link_format_matches_threaded_nodes(sid):
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    tn = threaded(scene)
    ln = links(scene)
    n = len(tn)
    n_leaves = sum(is_leaf(nd) for nd in tn)
    assert len(ln) == 2 * n + (n_leaves + 1) // 2
    boxes = ln[:2 * n].reshape(n, 8)[:, :6]
    assert np.array_equal(boxes.view(np.uint32), np.stack([nd["box"] for nd in tn]).view(np.uint32))
    w = ln.view(np.uint32)
    li = 0
    for k, nd in enumerate(tn):
        skip = int(nd["meta"]) & 0xFFFF
        miss = LEND if skip == END else 32 * skip
        assert int(w[2 * k + 1, 3]) == miss
        if is_leaf(nd):
            assert int(w[2 * k + 1, 2]) == LEAF | li << 16 | (0xFFFF if skip == END else 32 * skip)
            li += 1
        else:
            assert int(w[2 * k + 1, 2]) == 32 * (k + 1)


@pytest.mark.parametrize("sid", [0, 4, 6, 8])
def test_link_walk_replays_threaded_walk(sid):
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    tn = threaded(scene)
    ln = links(scene)
    rng = np.random.default_rng(sid)
    for p in (0.0, 0.3, 0.7, 1.0):
        for _ in range(20):
            hits = rng.random(len(tn)) < p
            assert walk_links(ln, len(tn), hits) == walk_threaded(tn, hits)


def heap_bvh(n_leaves):
    """A complete reference BVH (BVHNode std430 records) with n_leaves sphere leaves, heap order."""
    n_inner = n_leaves - 1
    rec = np.zeros(n_inner + n_leaves, dtype=[("box", "<f4", 6), ("l", "<i4"), ("r", "<i4")])
    rec["box"] = [-1, 1, -1, 1, -1, 1]
    for k in range(n_inner):
        rec[k]["l"], rec[k]["r"] = (2 * k + 1) << 16, (2 * k + 2) << 16
    for j in range(n_leaves):
        rec[n_inner + j]["l"] = rec[n_inner + j]["r"] = (j << 16) | 1
    return rec.tobytes()


@pytest.mark.parametrize("n_leaves,ok", [(1024, True), (1025, False)])
def test_link_format_needs_16_bit_offsets(n_leaves, ok):
    # 2 n_leaves - 1 threaded nodes; offsets of 32 B nodes fit 16 bits up to 2047 nodes
    L = rtamd.amd()
    b = heap_bvh(n_leaves)
    n = ctypes.c_int(-1)
    assert L.rt_debug_link_nodes(ctypes.create_string_buffer(b, len(b)), len(b), None, 0, ctypes.byref(n)) == 0
    assert (n.value > 0) == ok
