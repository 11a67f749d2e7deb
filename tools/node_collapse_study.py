#!/usr/bin/env python3
"""Which inner BVH nodes are worth testing at all?  CPU study for the link walk's node collapse.

A node whose box holds its children's boxes (boxes_nest) can be left out of the walk: where the
reference's test of it misses, the tests of its children (and theirs, down to the leaf nodes)
miss too -- the slab test is monotone in the box bounds and in ray_t.max -- so the leaves tested,
their order and ray_t are the reference's; only node tests change.  Leaving node N out saves its
V(N) tests and costs its two children V(N) - H(N) tests each (they are now tested wherever N was),
where H(N), the tests of N that hit, does not depend on what else is left out and V(N) = H of
N's nearest kept ancestor.  This tool logs the reference walk (oracle trace log) over sampled 8x8
tiles of the scene at 1080p, measures H per node, and prints the node tests per walk:
the reference tree, the best collapse for that sample (dynamic programme over the tree), and
the rules the host can apply without rays (surface-area ratio to the nearest kept ancestor).
usage: python tools/node_collapse_study.py [--scene 8] [--tiles 60] [--frames 4]
"""
import argparse
import ctypes
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "raytracing-book_amd"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402


def tree(scene):
    raw = scene.buffers[1]
    n = len(raw) // 32
    box = np.zeros((n, 6), np.float64)
    kids = {}
    for i in range(n):
        v = struct.unpack_from("<6f2i", raw, 32 * i)
        box[i] = v[:6]
        if (v[6] & 0xFFFF) == 0:
            kids[i] = ((v[7] >> 16) & 0xFFFF, (v[6] >> 16) & 0xFFFF)   # (right = tested first, left)
    return n, box, kids


def area(b):
    dx, dy, dz = b[1] - b[0], b[3] - b[2], b[5] - b[4]
    return 2.0 * (dx * dy + dy * dz + dz * dx)


def measure(scene, tiles, frames, seed=0):
    W, H = scene.width, scene.height
    n, box, kids = tree(scene)
    osc = pyoracle.OracleScene(scene, max_depth=5, spp=4096)
    L = pyoracle.lib()
    L.oracle_trace_log.restype = ctypes.c_long
    L.oracle_trace_log.argtypes = [ctypes.POINTER(pyoracle.OracleSceneDesc)] + [ctypes.c_int] * 8 + [
        ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32), ctypes.c_long]
    rng = np.random.default_rng(seed)
    rf = rtamd.frame_rand_factors(1, 0, frames)
    V = np.zeros(n, np.int64)
    Hh = np.zeros(n, np.int64)
    Hc = np.zeros(n, np.int64)   # camera rays only (bounce 0)
    walks = cwalks = 0
    for _ in range(tiles):
        tx, ty = int(rng.integers(0, W // 8)), int(rng.integers(0, H // 8))
        args = (ctypes.byref(osc.desc), W, H, tx * 8, tx * 8 + 8, ty * 8, ty * 8 + 8, 1, frames,
                rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        m = L.oracle_trace_log(*args, None, 0)
        buf = np.empty(m, dtype=np.int32)
        L.oracle_trace_log(*args, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), m)
        k = 0
        while k < m:
            cnt = buf[k + 3]
            cam = buf[k + 2] == 0
            seq = buf[k + 4:k + 4 + cnt]
            k += 4 + cnt
            walks += 1
            cwalks += cam
            idx = seq & 0x3FFFFFFF
            np.add.at(V, idx, 1)
            leaf_hit = (seq & 0x40000000) != 0
            hits = [int(i) for i in idx[leaf_hit]]
            for j in range(len(idx) - 1):
                c = kids.get(int(idx[j]))
                if c is not None and int(idx[j + 1]) == c[0]:
                    hits.append(int(idx[j]))
            np.add.at(Hh, hits, 1)
            if cam:
                np.add.at(Hc, hits, 1)
    measure.camera = (Hc, cwalks)
    return n, box, kids, V, Hh, walks


def cost(kids, Hh, walks, elim):
    """Node tests with the nodes in `elim` left out (V(N) = H of the nearest kept ancestor)."""
    total = 0
    stack = [(0, walks)]
    while stack:
        nd, v = stack.pop()
        if nd in elim:
            for c in kids[nd]:
                stack.append((c, v))
        else:
            total += v
            for c in kids.get(nd, ()):
                stack.append((c, Hh[nd]))
    return total


def best(kids, Hh, walks):
    """Dynamic programme: min node tests of N's subtree when N is reached V times (V one of the
    H values of N's ancestors, or the walks)."""
    memo = {}

    def f(nd, v):
        key = (nd, v)
        if key in memo:
            return memo[key]
        if nd not in kids:
            r = (v, False)
        else:
            keep = v + sum(f(c, int(Hh[nd]))[0] for c in kids[nd])
            drop = sum(f(c, v)[0] for c in kids[nd]) if nd != 0 else None
            r = (keep, False) if drop is None or keep <= drop else (drop, True)
        memo[key] = r
        return r

    sys.setrecursionlimit(100000)
    tot = f(0, walks)[0]
    elim = set()
    stack = [(0, walks)]
    while stack:
        nd, v = stack.pop()
        if nd not in kids:
            continue
        d = f(nd, v)[1]
        if d:
            elim.add(nd)
        for c in kids[nd]:
            stack.append((c, v if d else int(Hh[nd])))
    return tot, elim


def area_rule(kids, box, ratio):
    """Leave N out when its area is more than `ratio` of its nearest kept ancestor's."""
    elim = set()
    stack = [(0, None)]
    while stack:
        nd, anc = stack.pop()
        if nd not in kids:
            continue
        out = anc is not None and area(box[nd]) > ratio * area(box[anc])
        if out:
            elim.add(nd)
        for c in kids[nd]:
            stack.append((c, anc if out else nd))
    return elim


def camera_hits(scene, box, nx=240, ny=135):
    """Per node: how many of a grid of camera rays (pixel centres) hit its box in [0.001, inf) --
    the walk's hits with no prim test shrinking ray_t (what the host can count without shading)."""
    c = scene.camera.astype(np.float64)
    pos, ul, du, dv = c[4:7], c[8:11], c[12:15], c[16:19]
    W, H = scene.width, scene.height
    xs = (np.arange(nx) + 0.5) * W / nx
    ys = (np.arange(ny) + 0.5) * H / ny
    X, Y = np.meshgrid(xs, ys)
    d = ul[None, None, :] + X[..., None] * du + Y[..., None] * dv - pos
    d = d.reshape(-1, 3).astype(np.float32)
    o = pos.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = (np.float32(1.0) / d).astype(np.float32)
        hits = np.zeros(len(box), np.int64)
        for i, b in enumerate(box.astype(np.float32)):
            t0 = (b[[0, 2, 4]] - o) * inv
            t1 = (b[[1, 3, 5]] - o) * inv
            lo = np.maximum(np.float32(0.001), np.fmax.reduce(np.fmin(t0, t1), axis=1))
            hi = np.fmin.reduce(np.fmax(t0, t1), axis=1)
            hits[i] = int(np.count_nonzero(~(hi <= lo)))
    return hits, len(d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--tiles", type=int, default=60)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--spine", type=int, default=11)
    a = ap.parse_args()
    sc = rtamd.Scene(a.scene, 1920, 1080, seed=1)
    n, box, kids, V, Hh, walks = measure(sc, a.tiles, a.frames)
    base = cost(kids, Hh, walks, set())
    assert base == V.sum(), (base, V.sum())
    print(f"scene {a.scene}: {n} nodes ({len(kids)} inner), {walks} walks over {a.tiles} tiles x {a.frames} frames; "
          f"reference: {base / walks:.2f} node tests per walk")
    tot, elim = best(kids, Hh, walks)
    print(f"  best collapse for this sample: {tot / walks:.2f} per walk ({100 * (tot / base - 1):+.1f}%), "
          f"{len(elim)} inner nodes left out")
    for r in (0.5, 0.6, 0.7, 0.8, 0.9):
        e = area_rule(kids, box, r)
        c = cost(kids, Hh, walks, e)
        print(f"  area rule {r:.1f}: {c / walks:.2f} per walk ({100 * (c / base - 1):+.1f}%), {len(e)} left out")
    # the kernel already skips the spine (rt_capi.hip plan_spine: the first nodes of the right-most
    # chain, hits for a walk starting inside them; scene 8: 11): the gain over that
    chain, nd = [], 0
    while nd in kids and len(chain) < a.spine:
        chain.append(nd)
        nd = kids[nd][0]
    sp = cost(kids, Hh, walks, set(chain))
    print(f"  spine of {len(chain)} skipped (the kernel now): {sp / walks:.2f} per walk ({100 * (sp / base - 1):+.1f}%)")
    for r in (0.5, 0.7, 0.9):
        e = area_rule(kids, box, r) | set(chain)
        c = cost(kids, Hh, walks, e)
        print(f"  spine + area rule {r:.1f}: {c / walks:.2f} per walk ({100 * (c / sp - 1):+.1f}% vs the spine alone)")
    c = cost(kids, Hh, walks, elim | set(chain))
    print(f"  spine + best: {c / walks:.2f} per walk ({100 * (c / sp - 1):+.1f}% vs the spine alone)")
    Hc, cw = measure.camera
    _, ec = best(kids, Hc, cw)
    c = cost(kids, Hh, walks, ec | set(chain))
    print(f"  spine + best for the camera rays alone ({cw} walks): {c / walks:.2f} per walk "
          f"({100 * (c / sp - 1):+.1f}% vs the spine alone)")
    Hi, ni = camera_hits(sc, box)
    _, ei = best(kids, Hi, ni)
    c = cost(kids, Hh, walks, ei | set(chain))
    print(f"  spine + best for a 240x135 grid of camera rays, no prim tests ({len(ei)} left out): "
          f"{c / walks:.2f} per walk ({100 * (c / sp - 1):+.1f}% vs the spine alone)")
    # held-out check of the sample's own optimum on other tiles
    n2, _, _, V2, H2, w2 = measure(sc, a.tiles, a.frames, seed=1)
    b2 = cost(kids, H2, w2, set())
    c2 = cost(kids, H2, w2, elim)
    print(f"  the optimum on other tiles: {c2 / w2:.2f} per walk vs {b2 / w2:.2f} ({100 * (c2 / b2 - 1):+.1f}%)")


if __name__ == "__main__":
    main()
