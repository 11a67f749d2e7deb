"""Host-side tables of the exact near-first walk (rt_capi.hip build_fast,
RT_KERNEL_VARIANT=60), through rt_debug_fast_tables — no GPU needed.

* each of the 8 octant layouts is a threaded pre-order of one SAH tree that
  holds every solid prim of the reference BVH exactly once;
* every SAH box contains its children's boxes and the reference LEAF box of
  every prim below it (what the kernel's pruning argument relies on);
* opposite octants visit the leaves in opposite orders (near child first);
* ranks / leaf nodes follow the reference visit order, and the media slots
  of scene 8 are the fog (after its solid partner) and the
  subsurface medium, both tracked;
* scenes with rotated boxes (6, 7) are not eligible.
"""
import ctypes

import numpy as np
import pytest

import rtamd

DN = np.dtype([("box", "<f4", (6,)), ("meta", "<u4"), ("prims", "<u4")])
END = 0xFFFF
SPHERE, QUAD, MEDIUM, BOX = 1, 2, 3, 4
SOLID = (SPHERE, QUAD, BOX)


def buf(data):
    return ctypes.create_string_buffer(data, len(data)) if data else None


def threaded(scene):
    L = rtamd.amd()
    bvh = buf(scene.buffers[1])
    n = ctypes.c_int()
    assert L.rt_debug_threaded_bvh(bvh, len(scene.buffers[1]), None, 0, ctypes.byref(n)) == 0
    out = np.zeros(n.value, DN)
    assert L.rt_debug_threaded_bvh(bvh, len(scene.buffers[1]), out.ctypes.data, out.nbytes, ctypes.byref(n)) == 0
    return out


def fast_tables(scene):
    L = rtamd.amd()
    b = scene.buffers
    ns, nq, nb = len(b[0]) // 48, len(b[2]) // 80, len(b[4]) // 480
    per, nsl = ctypes.c_int(), ctypes.c_int()
    args = (buf(b[1]), len(b[1]), buf(b[2]), len(b[2]), buf(b[4]), len(b[4]), ns)
    rc = L.rt_debug_fast_tables(*args, None, 0, ctypes.byref(per), None, 0, None, ctypes.byref(nsl))
    assert rc in (0, 1)
    nodes = np.zeros(8 * max(per.value, 1), DN)
    info = np.zeros(max(ns + nq + nb, 1), np.uint32)
    slots = np.zeros((4, 4), np.int32)
    rc2 = L.rt_debug_fast_tables(*args, nodes.ctypes.data, nodes.nbytes, ctypes.byref(per),
                                 info.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), info.nbytes,
                                 slots.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.byref(nsl))
    assert rc2 == rc
    base = {SPHERE: 0, QUAD: ns, BOX: ns + nq}
    return rc, nodes[:8 * per.value].reshape(8, per.value), info[:ns + nq + nb], slots[:nsl.value], base


def leaf_slots(nd):
    m, p = int(nd["meta"]), int(nd["prims"])
    return [((m >> (16 + 4 * s)) & 0xF, (p >> (16 * s)) & 0xFFFF) for s in range(2)]


def is_leaf(nd):
    return (int(nd["meta"]) >> 16) & 0xF != 0


def inside(c, p):
    return c[0] >= p[0] and c[1] <= p[1] and c[2] >= p[2] and c[3] <= p[3] and c[4] >= p[4] and c[5] <= p[5]


def ref_solids(ref):
    """(type, idx) -> (rank, leaf) in the reference visit order (first slot wins)."""
    out, rank = {}, 0
    for k, nd in enumerate(ref):
        if not is_leaf(nd):
            continue
        for ty, ix in leaf_slots(nd):
            if ty in SOLID and (ty, ix) not in out:
                out[(ty, ix)] = (rank, k)
            rank += 1
    return out


@pytest.mark.parametrize("sid", [0, 1, 2, 3, 4, 5, 8, 9])
def test_layouts_hold_every_solid_once_inside_nested_boxes(sid):
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    ok, nodes, info, slots, base = fast_tables(scene)
    assert ok == 1
    ref = threaded(scene)
    solids = ref_solids(ref)
    for lay in nodes:
        n = len(lay)
        # an every-box-hit walk (inner -> next, leaf -> skip) visits 0..n-1 in order
        i, order = 0, []
        while i != END and len(order) <= n:
            order.append(i)
            i = int(lay[i]["meta"]) & 0xFFFF if is_leaf(lay[i]) else i + 1
        assert order == list(range(n))
        seen = []
        for k, nd in enumerate(lay):
            if is_leaf(nd):
                for ty, ix in leaf_slots(nd):
                    if ty:
                        seen.append((ty, ix))
                        leaf = solids[(ty, ix)][1]
                        assert inside(ref[leaf]["box"], nd["box"]), (k, ty, ix)
            else:
                c1 = k + 1
                c2 = int(lay[c1]["meta"]) & 0xFFFF
                assert c2 != END and c2 < n
                assert inside(lay[c1]["box"], nd["box"]) and inside(lay[c2]["box"], nd["box"])
        assert sorted(seen) == sorted(solids)
    for (ty, ix), (rank, leaf) in solids.items():
        assert int(info[base[ty] + ix]) == (rank << 16) | leaf


@pytest.mark.parametrize("sid", [0, 8])
def test_opposite_octants_visit_leaves_in_opposite_orders(sid):
    ok, nodes, *_ = fast_tables(rtamd.Scene(sid, 64, 36, seed=1))

    def leaves(lay):
        return [tuple(leaf_slots(nd)) for nd in lay if is_leaf(nd)]

    for o in range(8):
        assert leaves(nodes[o]) == leaves(nodes[7 - o])[::-1]
    assert leaves(nodes[0]) != leaves(nodes[1])


def test_scene8_media_slots():
    ok, nodes, info, slots, base = fast_tables(rtamd.Scene(8, 64, 36, seed=1))
    assert ok == 1 and len(slots) == 2
    ref = threaded(rtamd.Scene(8, 64, 36, seed=1))
    fog, sub = slots
    # the r = 5000 fog sorts last, so its 2-leaf (solid, fog) is the first leaf the reference visits
    first_leaf = next(k for k, nd in enumerate(ref) if is_leaf(nd))
    assert fog[1] == first_leaf and fog[2] == 0 and fog[3] == 2
    assert sub[2] == 1 and sub[1] > first_leaf
    # tracker bits mark exactly the subtrees holding solids ranked before each slot
    solids = ref_solids(ref)
    rank_of = {k: r for k, (r, _) in solids.items()}
    fog_rank = 1
    for lay in nodes:
        for nd in lay:
            if is_leaf(nd):
                early = any(ty and rank_of[(ty, ix)] < fog_rank for ty, ix in leaf_slots(nd))
                assert bool(int(nd["meta"]) & (1 << 24)) == early


@pytest.mark.parametrize("sid", [6, 7])
def test_rotated_boxes_take_the_exact_walk(sid):
    ok, *_ = fast_tables(rtamd.Scene(sid, 64, 36, seed=1))
    assert ok == 0
