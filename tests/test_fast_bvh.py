"""The non-parity fast mode's BVH (row f3; rt.h rt_set_bvh_mode RT_BVH_SAH, csrc/bvh_sah.h) —
host side, no GPU needed.

The SAH tree is built in the reference's own node format from the prims of the reference BVH's
leaves, so the oracle walks it unchanged: these tests check that it is a well-formed reference
BVH over exactly the same prims (media keep their reference leaf, hence their test multiplicity),
that the threaded / link formats the kernel walks accept it and replay its walk, and — with the
oracle — that it renders the same image statistically with far fewer node visits.  The GPU side
(tests/test_gpu_fast_bvh.py) checks the kernel on the SAH tree bit for bit against the oracle on
the same tree, and statistically against the reference BVH.
"""
import types

import numpy as np
import pytest

import pyoracle
import rtamd
from test_fast_tables import threaded
from test_link_nodes import check_layout, links_of, threaded_of, walk_links, walk_threaded

REC = np.dtype([("box", "<f4", 6), ("l", "<u4"), ("r", "<u4")])


def nodes(b):
    return np.frombuffer(b, REC)


def leaves(rec):
    return [(int(n["l"]), int(n["r"])) for n in rec if (int(n["l"]) & 0xFFFF) != 0]


def leaf_slots(rec):
    """Multiset of prim slots a walk tests, with the link format's rule: a singleton leaf
    tests a medium twice, anything else once (rt_capi.hip thread_bvh)."""
    out = {}
    for lo, r in leaves(rec):
        if lo == r and (lo & 0xFFFF) != 3:
            ids = [lo]
        else:
            ids = [lo, r]
        for p in ids:
            out[p] = out.get(p, 0) + 1
    return out


def with_bvh(sc, bvh):
    v = types.SimpleNamespace(**{k: getattr(sc, k) for k in ("textures", "camera", "background", "width", "height")})
    v.buffers = dict(sc.buffers)
    v.buffers[1] = bvh
    return v


@pytest.mark.parametrize("sid", range(10))
def test_sah_tree_is_a_reference_bvh_over_the_same_prims(sid):
    sc = rtamd.Scene(sid, 64, 36, seed=1)
    ref, sah = nodes(sc.buffers[1]), nodes(rtamd.sah_bvh(sc))
    # the same prims, each tested as often per walk (media keep their reference leaf)
    assert leaf_slots(sah) == leaf_slots(ref)
    med_ref = sorted(lv for lv in leaves(ref) if 3 in (lv[0] & 0xFFFF, lv[1] & 0xFFFF))
    med_sah = sorted(lv for lv in leaves(sah) if 3 in (lv[0] & 0xFFFF, lv[1] & 0xFFFF))
    assert med_ref == med_sah
    # a proper binary tree from node 0: every node reached once, inner nodes have two node
    # children whose boxes nest in the parent's, every prim inside its leaf's box
    seen, stack = set(), [0]
    while stack:
        k = stack.pop()
        assert k not in seen
        seen.add(k)
        n = sah[k]
        if (int(n["l"]) & 0xFFFF) == 0:
            assert (int(n["r"]) & 0xFFFF) == 0
            for c in (int(n["l"]) >> 16, int(n["r"]) >> 16):
                b, p = sah[c]["box"], n["box"]
                assert b[0] >= p[0] and b[1] <= p[1] and b[2] >= p[2] and b[3] <= p[3] and b[4] >= p[4] and b[5] <= p[5]
                stack.append(c)
    assert seen == set(range(len(sah)))
    assert sc.info["n_bvh_prims"] == len({p for lv in leaves(sah) for p in lv})
    # rt_set_bvh_mode's tree is this one (order 2 at the camera, prim cost 1)
    assert rtamd.sah_bvh(sc) == rtamd.sah_bvh(sc, 2, eye=sc.camera[4:7], prim_cost=1.0)


@pytest.mark.parametrize("sid", [0, 6, 7, 8])
def test_sah_tree_threads_and_link_walk_replays_it(sid):
    """The kernel's formats accept the SAH tree and replay its walk under random box hits."""
    sc = rtamd.Scene(sid, 64, 36, seed=1)
    b = rtamd.sah_bvh(sc)
    tn = threaded_of(b)
    ln = links_of(b)
    order = check_layout(tn, ln)
    rng = np.random.default_rng(sid)
    for p in (0.3, 0.7, 1.0):
        for _ in range(10):
            hits = rng.random(len(tn)) < p
            assert walk_links(ln, len(tn), hits, order) == walk_threaded(tn, hits)
    assert len(threaded(sc)) == len(nodes(sc.buffers[1]))


def test_sah_builder_rejects_bad_input():
    sc = rtamd.Scene(8, 64, 36, seed=1)
    bad = bytearray(sc.buffers[1])
    # a leaf pointing at a sphere index past the records
    rec = np.frombuffer(bad, REC).copy()
    k = next(i for i, n in enumerate(rec) if (int(n["l"]) & 0xFFFF) == 1)
    rec[k]["l"] = (60000 << 16) | 1
    v = with_bvh(sc, rec.tobytes())
    with pytest.raises(rtamd.RTError):
        rtamd.sah_bvh(v)
    with pytest.raises(rtamd.RTError):
        rtamd.sah_bvh(sc, prim_cost=0.0)


@pytest.mark.parametrize("sid,max_visit_ratio", [(8, 0.55), (0, 0.8)])
def test_sah_tree_renders_the_same_image_with_fewer_visits(sid, max_visit_ratio):
    """The oracle on both trees at equal samples: the same image statistically (the per-pixel
    sample streams differ only where a medium's rand() draw moves in the visit sequence, or a
    tie resolves another way), far fewer node visits and no more prim tests.  Scene 8 (fog
    everywhere) differs per pixel; scene 0 (no media) only by exact ties."""
    W, H, F = 96, 54, 16
    sc = rtamd.Scene(sid, W, H, seed=1)
    rf = rtamd.frame_rand_factors(1, 0, F)
    out = {}
    for name, b in (("ref", sc.buffers[1]), ("sah", rtamd.sah_bvh(sc))):
        img, c = pyoracle.render(pyoracle.OracleScene(with_bvh(sc, b), max_depth=5, spp=4096), rf, nthreads=4,
                                 counters=True)
        n = c["samples"]
        out[name] = (img, c["node_visits"] / n,
                     (c["sphere_tests"] + c["box_tests"] + c["quad_tests"] + c["medium_tests"]) / n)
    (ri, rv, rt), (si, sv, st) = out["ref"], out["sah"]
    assert sv <= max_visit_ratio * rv, (sv, rv)
    assert st <= rt * 1.001, (st, rt)
    rm, sm = np.nanmean(ri[..., :3], axis=(0, 1)), np.nanmean(si[..., :3], axis=(0, 1))
    assert np.all(np.abs(sm / rm - 1.0) < 0.03), (sm, rm)
    if sid == 0:   # no medium: the same hits, so nearly every pixel identical
        same = np.all(ri.view(np.uint32) == si.view(np.uint32), axis=-1).mean()
        assert same > 0.99, same
