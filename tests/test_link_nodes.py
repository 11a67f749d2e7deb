"""The link-format BVH the default kernel walks (rt_capi.hip build_links,
rt_device.h RT_LINK_*; rt_kernel.hip link_walk) — host-side, no GPU needed.

Every node keeps its threaded node's box and is placed breadth-first (the
root's level first, an inner node's right child before its left one), so a
two-level launch stages the top levels every ray walks as one LDS prefix.
Its hit / miss words are the threaded walk's successors as byte addresses; a
hit leaf leaves the loop with its leaf ordinal, and the leaf's record holds its
prim types and the address the walk continues at.  Under any pattern of box
hits the link walk visits the same nodes and tests the same leaves, in the same
order, as the threaded walk (which itself replays the reference's stack walk,
test_abi.py) — for the shipped scenes and for BVHs up to the reference's 16-bit
limit of 65535 nodes (the round-2 format stopped at 2047).
"""
import ctypes

import numpy as np
import pytest

import rtamd
from test_fast_tables import END, is_leaf, threaded

LEAF, LEND, NEXT_END = 0x80000000, 0xFFFFFFFF, 0xFFFFFF


def links_of(bvh_bytes):
    L = rtamd.amd()
    bvh = ctypes.create_string_buffer(bvh_bytes, len(bvh_bytes))
    n = ctypes.c_int()
    assert L.rt_debug_link_nodes(bvh, len(bvh_bytes), None, 0, ctypes.byref(n)) == 0
    out = np.zeros((max(n.value, 1), 4), np.float32)
    assert L.rt_debug_link_nodes(bvh, len(bvh_bytes), out.ctypes.data, out.nbytes, ctypes.byref(n)) == 0
    return out[:n.value]


def threaded_of(bvh_bytes):
    L = rtamd.amd()
    n = ctypes.c_int()
    assert L.rt_debug_threaded_bvh(bvh_bytes, len(bvh_bytes), None, 0, ctypes.byref(n)) == 0
    from test_fast_tables import DN
    out = np.zeros(n.value, DN)
    assert L.rt_debug_threaded_bvh(bvh_bytes, len(bvh_bytes), out.ctypes.data, out.nbytes, ctypes.byref(n)) == 0
    return out


def bfs_order(tn):
    """Breadth-first order of the threaded nodes: an inner node k's children are its
    right child k + 1 and its left child skip(k + 1)."""
    order, h = [0], 0
    while h < len(order):
        k = order[h]
        h += 1
        if not is_leaf(tn[k]):
            order += [k + 1, int(tn[k + 1]["meta"]) & 0xFFFF]
    return order


def walk_threaded(tn, hits):
    i, seen, tested = 0, [], []
    while i != END:
        seen.append(i)
        nd = tn[i]
        skip = int(nd["meta"]) & 0xFFFF
        if not hits[i]:
            i = skip
        elif is_leaf(nd):
            tested.append((int(nd["meta"]) >> 16 & 0xFF, int(nd["prims"])))
            i = skip
        else:
            i += 1
    return seen, tested


def walk_links(ln, n, hits, node_of_slot):
    """The kernel's loop (render_stream): nodes by address, leaves by ordinal."""
    words = ln.view(np.uint32)
    leaves = words[2 * n:].reshape(-1, 2)
    nx, seen, tested = 0, [], []
    while True:
        while nx < LEAF:
            k = node_of_slot[nx // 32]
            seen.append(k)
            nx = int(words[2 * (nx // 32) + 1, 2] if hits[k] else words[2 * (nx // 32) + 1, 3])
        if nx == LEND:
            break
        lf = leaves[nx & 0x7FFFFFFF]
        tested.append((int(lf[0]) & 0xFF, int(lf[1])))
        nx = int(lf[0]) >> 8
        if nx == NEXT_END:
            break
    return seen, tested


def check_layout(tn, ln):
    n = len(tn)
    order = bfs_order(tn)
    assert sorted(order) == list(range(n))
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    n_leaves = sum(is_leaf(nd) for nd in tn)
    assert len(ln) == 2 * n + (n_leaves + 1) // 2
    boxes = ln[:2 * n].reshape(n, 8)[:, :6]
    assert np.array_equal(boxes.view(np.uint32), np.stack([tn[k]["box"] for k in order]).view(np.uint32))
    w = ln.view(np.uint32)
    leaves = w[2 * n:].reshape(-1, 2)
    li = 0
    for k, nd in enumerate(tn):
        skip = int(nd["meta"]) & 0xFFFF
        at = 2 * pos[k] + 1
        assert int(w[at, 3]) == (LEND if skip == END else 32 * pos[skip])
        if is_leaf(nd):
            assert int(w[at, 2]) == LEAF | li
            assert int(leaves[li, 0]) == (int(nd["meta"]) >> 16 & 0xFF) | (NEXT_END if skip == END else 32 * pos[skip]) << 8
            assert int(leaves[li, 1]) == int(nd["prims"])
            li += 1
        else:
            assert int(w[at, 2]) == 32 * pos[k + 1]
    return order


@pytest.mark.parametrize("sid", range(10))
def test_link_format_matches_threaded_nodes(sid):
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    check_layout(threaded(scene), links_of(scene.buffers[1]))


@pytest.mark.parametrize("sid", [0, 4, 6, 8])
def test_link_walk_replays_threaded_walk(sid):
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    tn = threaded(scene)
    ln = links_of(scene.buffers[1])
    order = check_layout(tn, ln)
    rng = np.random.default_rng(sid)
    for p in (0.0, 0.3, 0.7, 1.0):
        for _ in range(20):
            hits = rng.random(len(tn)) < p
            assert walk_links(ln, len(tn), hits, order) == walk_threaded(tn, hits)


def heap_bvh(n_leaves):
    """A complete reference BVH (BVHNode std430 records) with n_leaves sphere leaves, heap order."""
    n_inner = n_leaves - 1
    rec = np.zeros(n_inner + n_leaves, dtype=[("box", "<f4", 6), ("l", "<u4"), ("r", "<u4")])
    rec["box"] = [-1, 1, -1, 1, -1, 1]
    for k in range(n_inner):
        rec[k]["l"], rec[k]["r"] = (2 * k + 1) << 16, (2 * k + 2) << 16
    for j in range(n_leaves):
        rec[n_inner + j]["l"] = rec[n_inner + j]["r"] = (j << 16) | 1
    return rec.tobytes()


@pytest.mark.parametrize("n_leaves", [1024, 1025, 4096, 32768])
def test_link_format_reaches_the_16_bit_node_limit(n_leaves):
    """Up to 2 * 32768 - 1 = 65535 nodes (the reference's 16-bit node indices)."""
    b = heap_bvh(n_leaves)
    tn = threaded_of(b)
    ln = links_of(b)
    assert len(tn) == 2 * n_leaves - 1 and len(ln) > 0
    order = check_layout(tn, ln)
    if n_leaves <= 4096:
        rng = np.random.default_rng(n_leaves)
        for p in (0.5, 0.9, 1.0):
            hits = rng.random(len(tn)) < p
            assert walk_links(ln, len(tn), hits, order) == walk_threaded(tn, hits)


# ---- box pre-test nodes (option box_vnodes, round 5) -------------------------------------------
PRETESTED = 8


def vnode_links(bvh_bytes, vbox):
    L = rtamd.amd()
    bvh = ctypes.create_string_buffer(bvh_bytes, len(bvh_bytes))
    vb = np.ascontiguousarray(vbox, np.float32)
    n, nn = ctypes.c_int(), ctypes.c_int()
    fp = vb.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert L.rt_debug_link_nodes_vbox(bvh, len(bvh_bytes), fp, len(vb) // 6, None, 0, ctypes.byref(n),
                                      ctypes.byref(nn)) == 0
    out = np.zeros((max(n.value, 1), 4), np.float32)
    assert L.rt_debug_link_nodes_vbox(bvh, len(bvh_bytes), fp, len(vb) // 6, out.ctypes.data, out.nbytes,
                                      ctypes.byref(n), ctypes.byref(nn)) == 0
    return out[:n.value], nn.value


def walk_links_n(ln, n_all, hits_of_slot):
    """The kernel's loop over links with n_all nodes; hits_of_slot[address // 32] -> bool."""
    words = ln.view(np.uint32)
    leaves = words[2 * n_all:].reshape(-1, 2)
    nx, tested = 0, []
    while True:
        while nx < LEAF:
            nx = int(words[2 * (nx // 32) + 1, 2] if hits_of_slot[nx // 32] else words[2 * (nx // 32) + 1, 3])
        if nx == LEND:
            break
        lf = leaves[nx & 0x7FFFFFFF]
        tested.append((int(lf[0]) & 0xFF, int(lf[1])))
        nx = int(lf[0]) >> 8
        if nx == NEXT_END:
            break
    return tested


@pytest.mark.parametrize("sid", [8, 7, 6, 4])
def test_box_pretest_nodes_replay_the_walk(sid):
    """The walk over the links with box pre-test nodes tests, under any pattern of box hits, the
    threaded walk's prims in the same order, except that a box whose pre-test node misses is
    skipped -- exactly what the leaf stage's pre-test did -- and each box of an all-box leaf is its
    own record, marked pre-tested.  Other leaves are unchanged."""
    scene = rtamd.Scene(sid, 64, 36, seed=1)
    tn = threaded(scene)
    n = len(tn)
    nb = len(scene.buffers[4]) // 480
    vbox = np.random.default_rng(sid).random(6 * max(nb, 1)).astype(np.float32)[:6 * nb]
    ln, n_all = vnode_links(scene.buffers[1], vbox)
    plain = links_of(scene.buffers[1])
    order = check_layout(tn, plain)
    # the tree's nodes keep their boxes and places; chain nodes follow, one per box of an all-box leaf,
    # in threaded order, holding that box's bounds
    assert np.array_equal(ln[:2 * n].reshape(n, 8)[:, :6].view(np.uint32), plain[:2 * n].reshape(n, 8)[:, :6].view(np.uint32))
    chain = []
    for k, nd in enumerate(tn):
        t0, t1 = (int(nd["meta"]) >> 16) & 0xF, (int(nd["meta"]) >> 20) & 0xF
        if is_leaf(nd) and t0 == 4 and t1 in (0, 4):
            chain += [(k, int(nd["prims"]) & 0xFFFF)] + ([(k, int(nd["prims"]) >> 16)] if t1 else [])
    assert n_all == n + len(chain)
    for j, (_, b) in enumerate(chain):
        assert np.array_equal(ln[2 * (n + j)][:4], vbox[6 * b:6 * b + 4]) and np.array_equal(ln[2 * (n + j) + 1][:2],
                                                                                           vbox[6 * b + 4:6 * b + 6])
    first = {}
    for j, (k, _) in enumerate(chain):
        first.setdefault(k, n + j)
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    rng = np.random.default_rng(100 + sid)
    for p in (0.3, 0.7, 1.0):
        for _ in range(20):
            hits = rng.random(n) < p
            vh = rng.random(max(len(chain), 1)) < 0.5
            slot_hits = np.zeros(n_all, bool)
            slot_hits[pos] = hits
            slot_hits[n:] = vh[:len(chain)]
            want = []
            for types, prims in walk_threaded(tn, hits)[1]:
                k = None
                if types & 0xF == 4 and (types >> 4) in (0, 4):
                    k = next(kk for kk in first if int(tn[kk]["prims"]) == prims and is_leaf(tn[kk]))
                if k is None:
                    want.append((types, prims))
                    continue
                boxes = [prims & 0xFFFF] + ([prims >> 16] if types >> 4 else [])
                for j, b in enumerate(boxes):
                    if slot_hits[first[k] + j]:
                        want.append((4 | PRETESTED, b))
            assert walk_links_n(ln, n_all, slot_hits) == want


# ---- node collapse (option collapse, round 5) ------------------------------------------------------
def collapse_links(scene, width=1920, height=1080, cam=None, rebuild=0):
    L = rtamd.amd()
    b = scene.buffers[1]
    bvh = ctypes.create_string_buffer(b, len(b))
    cam = np.ascontiguousarray(scene.camera if cam is None else cam, np.float32)
    n, nd = ctypes.c_int(), ctypes.c_int()
    assert L.rt_debug_collapse_links(bvh, len(b), cam.ctypes.data, width, height, rebuild, None, 0, ctypes.byref(n),
                                     None, 0, ctypes.byref(nd)) == 0
    out = np.zeros((max(n.value, 1), 4), np.float32)
    m = len(b) // 32
    drop = np.zeros(m, np.uint8)
    assert L.rt_debug_collapse_links(bvh, len(b), cam.ctypes.data, width, height, rebuild, out.ctypes.data,
                                     out.nbytes, ctypes.byref(n), drop.ctypes.data, drop.nbytes,
                                     ctypes.byref(nd)) == 0
    return out[:n.value], drop, nd.value


def nested_hits(tn, rng, p):
    """A random box-hit pattern in which a node hits only where its parent does (boxes nest, and the
    slab test is monotone in the box: rt_capi.hip plan_collapse)."""
    hits = np.zeros(len(tn), bool)
    hits[0] = rng.random() < max(p, 0.5)
    for k, nd in enumerate(tn):
        if is_leaf(nd):
            continue
        for c in (k + 1, int(tn[k + 1]["meta"]) & 0xFFFF):
            hits[c] = hits[k] and rng.random() < p
    return hits


@pytest.mark.parametrize("sid", [8, 0, 6, 7, 4])
def test_collapsed_walk_tests_the_same_leaves(sid):
    """Leaving out inner nodes (option collapse): under every nested pattern of box hits the walk
    over the collapsed links tests the threaded walk's leaves in the same order, with fewer or more
    node tests.  The kept nodes keep their breadth-first order and boxes, the left-out ones get no
    place; the root and the leaf nodes are never left out."""
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    tn = threaded(scene)
    n = len(tn)
    ln, drop, nd = collapse_links(scene)
    plain = links_of(scene.buffers[1])
    check_layout(tn, plain)
    assert nd == int(drop.sum())
    assert drop[0] == 0 and not any(drop[k] for k in range(n) if is_leaf(tn[k]))
    order = [k for k in bfs_order(tn) if not drop[k]]
    nk = len(order)
    n_leaves = sum(is_leaf(x) for x in tn)
    assert nk == n - nd and len(ln) == 2 * nk + (n_leaves + 1) // 2
    assert np.array_equal(ln[:2 * nk].reshape(nk, 8)[:, :6].view(np.uint32),
                          np.stack([tn[k]["box"] for k in order]).view(np.uint32))
    n = nk
    if sid == 8:
        assert nd > 100   # the fog's chain and much of the sphere cluster's upper levels
    rng = np.random.default_rng(200 + sid)
    steps_full = steps_coll = 0
    for p in (0.3, 0.6, 0.9, 1.0):
        for _ in range(25):
            hits = nested_hits(tn, rng, p)
            seen, want = walk_threaded(tn, hits)
            s2, got = walk_links(ln, n, hits, order)
            assert got == want
            assert not any(drop[k] for k in s2)   # a left-out node is never reached
            steps_full += len(seen)
            steps_coll += len(s2)
    assert steps_coll != steps_full or nd == 0


@pytest.mark.parametrize("rebuild", [0, 1, 2])
def test_collapse_keeps_a_tree_whose_boxes_do_not_nest(rebuild):
    """No collapse unless every child box lies inside its parent's (boxes_nest) and no box is flat;
    and no inner-node rebuild either: over a tree whose boxes do not nest the
    reference's walk prunes leaves at a missed ancestor that a rebuilt tree would reach, so the
    walk keeps the uploaded tree's links exactly."""
    rec = np.frombuffer(heap_bvh(64), dtype=[("box", "<f4", 6), ("l", "<u4"), ("r", "<u4")]).copy()
    rec[5]["box"] = [-2, 2, -1, 1, -1, 1]   # an inner node wider than its parent
    scene = rtamd.Scene(9, 64, 36, seed=1)
    scene.buffers = dict(scene.buffers)
    scene.buffers[1] = rec.tobytes()
    links, drop, nd = collapse_links(scene, rebuild=rebuild)
    assert nd == 0 and not drop.any()
    assert np.array_equal(links.view(np.uint32), links_of(rec.tobytes()).view(np.uint32))
    # the nesting tree is rebuilt (the gate is the nesting, not the size)
    if rebuild:
        ok = np.frombuffer(heap_bvh(64), dtype=rec.dtype).copy()
        ok["box"][63:] = [[-1 + j / 64, -1 + (j + 1) / 64, -1, 1, -1, 1] for j in range(64)]
        links2, _, _ = collapse_links(scene_with_bvh(scene, ok.tobytes()), rebuild=rebuild)
        assert not np.array_equal(links2.view(np.uint32), links_of(ok.tobytes()).view(np.uint32))


def scene_with_bvh(scene, b):
    scene.buffers = dict(scene.buffers)
    scene.buffers[1] = b
    return scene


# ---- inner-node rebuild (option rebuild, round 5) -------------------------------------------------
def slab_hit(b, o, inv, tmin, tmax, exact):
    """The kernel's node test on float32 values: the NaN-ignoring min / max form (aabb_pk), or, for
    a ray with a -inf component of 1/dir, the reference's per-axis slab (rt_kernel_common.h slab)."""
    t0 = (np.float32(b[0::2]) - o) * inv
    t1 = (np.float32(b[1::2]) - o) * inv
    if not exact:
        lo = np.fmax(np.float32(tmin), np.fmax.reduce(np.fmin(t0, t1)))
        hi = np.fmin(np.float32(tmax), np.fmin.reduce(np.fmax(t0, t1)))
        return not (hi <= lo)
    lo, hi = np.float32(tmin), np.float32(tmax)
    for k in range(3):
        ordr = t0[k] < t1[k]
        a, c = (t0[k], t1[k]) if ordr else (t1[k], t0[k])
        lo = a if a > lo else lo
        hi = c if c < hi else hi
    return not (hi <= lo)


def shrink(prims, o, d, tmax, box):
    """A leaf's tests as the walks see them: deterministic in (leaf, ray, ray_t.max) -- some leaves
    'hit' at the distance to their box centre when it is closer than ray_t.max."""
    if hash(int(prims)) % 3:
        return tmax
    c = np.float32([(box[0] + box[1]) / 2, (box[2] + box[3]) / 2, (box[4] + box[5]) / 2])
    t = np.float32(np.dot(c - o, d) / max(np.dot(d, d), np.float32(1e-30)))
    return t if 0.001 < t < tmax else tmax


def walk_tree_rays(tn, o, d, inv, exact):
    i, tmax, tested = 0, np.float32(np.inf), []
    while i != END:
        nd = tn[i]
        skip = int(nd["meta"]) & 0xFFFF
        if not slab_hit(nd["box"], o, inv, 0.001, tmax, exact):
            i = skip
        elif is_leaf(nd):
            tested.append((int(nd["prims"]), float(tmax)))
            tmax = shrink(nd["prims"], o, d, tmax, nd["box"])
            i = skip
        else:
            i += 1
    return tested


def walk_links_rays(ln, n, o, d, inv, exact):
    words = ln.view(np.uint32)
    leaves = words[2 * n:].reshape(-1, 2)
    nx, tmax, tested = 0, np.float32(np.inf), []
    last_box = None
    while True:
        while nx < LEAF:
            at = nx // 32
            box = np.concatenate([ln[2 * at], ln[2 * at + 1][:2]])
            h = slab_hit(box, o, inv, 0.001, tmax, exact)
            if h:
                last_box = box
            nx = int(words[2 * at + 1, 2] if h else words[2 * at + 1, 3])
        if nx == LEND:
            break
        lf = leaves[nx & 0x7FFFFFFF]
        tested.append((int(lf[1]), float(tmax)))
        tmax = shrink(lf[1], o, d, tmax, last_box)
        nx = int(lf[0]) >> 8
        if nx == NEXT_END:
            break
    return tested


@pytest.mark.parametrize("rebuild", [1, 2])
@pytest.mark.parametrize("sid", [8, 0, 6])
def test_rebuilt_inner_nodes_test_the_same_leaves(sid, rebuild):
    """The inner nodes rebuilt over the reference's leaf sequence (option rebuild: 1 greedy surface-area
    splits, 2 the least summed inner-box area by a dynamic programme), then collapsed
    (option collapse): for rays through the scene -- some with a zero direction component (1/dir
    = +-inf), ray_t.max shrinking at some leaves -- the walk over the links tests the reference
    tree's leaves in the same order under the same ray_t.max.  Nothing about the inner nodes
    matters but that their boxes hold the leaves' (rt_capi.hip rebuild_inner)."""
    scene = rtamd.Scene(sid, 1920, 1080, seed=1)
    tn = threaded(scene)
    n = len(tn)
    ln, drop, nd = collapse_links(scene, rebuild=rebuild)
    nk = n - nd   # the nodes with a place in the links (left-out ones have none)
    leaves_tn = [(int(x["meta"]) >> 16 & 0xFF, int(x["prims"])) for x in tn if is_leaf(x)]
    w = ln.view(np.uint32)
    assert len(ln) == 2 * nk + (len(leaves_tn) + 1) // 2
    rec = [(int(a) & 0xFF, int(b)) for a, b in w[2 * nk:].reshape(-1, 2)][:len(leaves_tn)]
    assert rec == leaves_tn   # the same leaf records, in the same order
    boxes = np.stack([x["box"] for x in tn])
    lo, hi = boxes[0, 0::2], boxes[0, 1::2]
    lo, hi = np.maximum(lo, -600), np.minimum(hi, 600)
    rng = np.random.default_rng(300 + sid)
    cam = scene.camera[4:7].astype(np.float32)
    differ = 0
    for r in range(300):
        o = cam if r % 3 == 0 else (lo + (hi - lo) * rng.random(3)).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        if r % 7 == 0:
            d[rng.integers(3)] = 0.0
        if r % 11 == 0:
            d[rng.integers(3)] = -0.0
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            inv = (np.float32(1.0) / d).astype(np.float32)
            exact = bool(np.any(inv == -np.inf))
            want = walk_tree_rays(tn, o, d, inv, exact)
            got = walk_links_rays(ln, nk, o, d, inv, exact)
        assert got == want, (r, o, d)
        differ += len(want) > 0
    assert differ > 50


@pytest.mark.parametrize("rebuild", [1, 2])
def test_rebuilt_inner_nodes_of_a_4000_sphere_cloud(rebuild):
    """The same replay on the ~4000-node cloud (tests/adversarial.py): about 2000 leaves, so the
    dynamic programme runs with its Knuth window over a long sequence (rebuild=2)."""
    import adversarial
    scene = adversarial.sphere_cloud(4000, 4)
    tn = threaded(scene)
    n = len(tn)
    ln, drop, nd = collapse_links(scene, 64, 48, rebuild=rebuild)
    nk = n - nd
    rng = np.random.default_rng(400 + rebuild)
    boxes = np.stack([x["box"] for x in tn])
    lo, hi = boxes[0, 0::2], boxes[0, 1::2]
    cam = scene.camera[4:7].astype(np.float32)
    hits = 0
    for r in range(120):
        o = cam if r % 2 == 0 else (lo + (hi - lo) * rng.random(3)).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        if r % 9 == 0:
            d[rng.integers(3)] = 0.0
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            inv = (np.float32(1.0) / d).astype(np.float32)
            exact = bool(np.any(inv == -np.inf))
            want = walk_tree_rays(tn, o, d, inv, exact)
            got = walk_links_rays(ln, nk, o, d, inv, exact)
        assert got == want, r
        hits += len(want) > 0
    assert hits > 20
