"""Analysis (test infrastructure, not collected by pytest): SIMD schedule
simulator for the render kernel's wave (one 8x8 tile = 64 lanes), replaying
the oracle's exact per-lane traversal logs (node pops, leaf hits).

Schedules:
  A  bounce-synchronous while-while (the round-1 kernel): every lane traces its
     j-th ray together; node steps run until each unfinished lane has a leaf
     pending, then one leaf stage; after the wave's longest trace, one shading
     stage for all lanes.
  B  decoupled: a lane whose trace finished waits in a shade queue while the
     others keep traversing; the shading stage runs once >= K lanes wait (or
     nothing else can run), then those lanes start their next ray at once.

Stage costs (wave-iterations) are calibrated on schedule A against the stats
build's measured split (node 48 %, leaf 35 %, shade 12.6 %) and then
used to predict B.
usage: python tests/analysis/simd_schedule.py [--scene 8] [--tiles 24] [--frames 8]
"""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

LEAF = 0x40000000


def lane_traces(buf):
    """pixel -> list of traces (in frame/bounce order); trace = list of (node, leaf_hit)."""
    out = {}
    k = 0
    while k < len(buf):
        pix, fr, b, m = buf[k:k + 4]
        seq = buf[k + 4:k + 4 + m]
        out.setdefault(int(pix), []).append(((seq & LEAF) != 0))
        k += 4 + m
    return out


def run_trace_set(traces):
    """While-while over one set of concurrent traces (one per lane); returns
    (node_iters, node_lanes, leaf_iters, leaf_lanes, steps_per_lane)."""
    n = len(traces)
    ptr = np.zeros(n, int)
    ln = np.array([len(t) for t in traces])
    pend = np.zeros(n, bool)
    ni = nl = li = ll = 0
    while True:
        while True:
            act = (ptr < ln) & ~pend
            c = int(act.sum())
            if c == 0:
                break
            ni += 1
            nl += c
            idx = np.nonzero(act)[0]
            for i in idx:
                if traces[i][ptr[i]]:
                    pend[i] = True
                ptr[i] += 1
        if not pend.any():
            break
        li += 1
        ll += int(pend.sum())
        pend[:] = False
    return ni, nl, li, ll


def schedule_a(lanes):
    tot = np.zeros(6)
    depth = max(len(t) for t in lanes)
    for j in range(depth):
        cur = [t[j] for t in lanes if j < len(t)]
        ni, nl, li, ll = run_trace_set(cur)
        tot += [ni, nl, li, ll, 1, len(cur)]
    return tot   # node_it, node_ln, leaf_it, leaf_ln, shade_it, shade_ln


def schedule_b(lanes, K):
    n = len(lanes)
    tr = [0] * n                     # index of the lane's current trace
    ptr = np.zeros(n, int)
    pend = np.zeros(n, bool)
    state = np.zeros(n, int)         # 0 traversing, 1 waiting to shade, 2 done
    for i in range(n):
        if not lanes[i]:
            state[i] = 2
    ni = nl = li = ll = si = sl = 0
    while (state != 2).any():
        trav = state == 0
        while True:
            act = trav & ~pend
            for i in np.nonzero(act)[0]:
                if ptr[i] >= len(lanes[i][tr[i]]):
                    act[i] = False
                    state[i] = 1
                    trav[i] = False
            c = int(act.sum())
            if c == 0:
                break
            ni += 1
            nl += c
            for i in np.nonzero(act)[0]:
                if lanes[i][tr[i]][ptr[i]]:
                    pend[i] = True
                ptr[i] += 1
        if pend.any():
            li += 1
            ll += int(pend.sum())
            pend[:] = False
            for i in np.nonzero(trav)[0]:   # lanes whose trace ended with that leaf
                if ptr[i] >= len(lanes[i][tr[i]]):
                    state[i] = 1
        waiting = state == 1
        if waiting.sum() >= K or (not (state == 0).any() and waiting.any()):
            si += 1
            sl += int(waiting.sum())
            for i in np.nonzero(waiting)[0]:
                tr[i] += 1
                ptr[i] = 0
                state[i] = 0 if tr[i] < len(lanes[i]) else 2
    return np.array([ni, nl, li, ll, si, sl], float)


def schedule_s(lanes, K, Q, stop="all"):
    """Speculative walk (leaves queued, up to Q per lane; inner nodes may be
    tested with a stale ray_t.max, leaves re-tested exactly when popped) plus
    decoupled shading at >= K waiting lanes.  Node sequences are the exact
    ones (the stale-tmax superset is not modelled)."""
    n = len(lanes)
    tr = [0] * n
    ptr = np.zeros(n, int)
    q = np.zeros(n, int)              # queued leaves
    state = np.zeros(n, int)          # 0 traversing, 1 waiting to shade, 2 done
    for i in range(n):
        if not lanes[i]:
            state[i] = 2
    ni = nl = li = ll = si = sl = 0
    while (state != 2).any():
        while True:
            trav = state == 0
            walking = trav & (ptr < np.array([len(lanes[i][tr[i]]) if state[i] != 2 else 0 for i in range(n)]))
            if stop == "all":   # step until every traversing lane has a leaf queued or finished walking
                need = walking & (q == 0)
            else:
                need = walking & (q < Q)
            if not need.any():
                break
            act = walking & (q < Q)
            ni += 1
            nl += int(act.sum())
            for i in np.nonzero(act)[0]:
                if lanes[i][tr[i]][ptr[i]]:
                    q[i] += 1
                ptr[i] += 1
        if (q > 0).any():
            li += 1
            ll += int((q > 0).sum())
            q[q > 0] -= 1
        for i in range(n):
            if state[i] == 0 and q[i] == 0 and ptr[i] >= len(lanes[i][tr[i]]):
                state[i] = 1
        waiting = state == 1
        if waiting.sum() >= K or (not (state == 0).any() and waiting.any()):
            si += 1
            sl += int(waiting.sum())
            for i in np.nonzero(waiting)[0]:
                tr[i] += 1
                ptr[i] = 0
                state[i] = 0 if tr[i] < len(lanes[i]) else 2
    return np.array([ni, nl, li, ll, si, sl], float)


def schedule_fetch(pool, R, Q=1, lanes_n=64):
    """Trace-only wavefront schedule with dynamic ray fetch: every trace in
    `pool` (list of traces, each a list of leaf-hit flags per node) is walked by
    one lane; lanes whose trace ended are refilled from the pool once >= R lanes
    are idle (or when the wave would otherwise stall).  While-while walk with a
    leaf queue of depth Q (Q=1: no speculation).  Returns node/leaf iteration
    and lane counts."""
    it = iter(pool)
    cur = [None] * lanes_n
    ptr = [0] * lanes_n
    q = [0] * lanes_n
    ni = nl = li = ll = 0
    exhausted = False

    def refill():
        nonlocal exhausted
        for k in range(lanes_n):
            if cur[k] is None and not exhausted:
                t = next(it, None)
                if t is None:
                    exhausted = True
                else:
                    cur[k] = t
                    ptr[k] = 0
                    q[k] = 0
    refill()
    while any(c is not None for c in cur):
        # node steps
        while True:
            walking = [c is not None and ptr[k] < len(c) for k, c in enumerate(cur)]
            need = [walking[k] and q[k] == 0 for k in range(lanes_n)]
            if not any(need):
                break
            act = [walking[k] and q[k] < Q for k in range(lanes_n)]
            ni += 1
            nl += sum(act)
            for k in range(lanes_n):
                if act[k]:
                    if cur[k][ptr[k]]:
                        q[k] += 1
                    ptr[k] += 1
        pend = [q[k] > 0 for k in range(lanes_n)]
        if any(pend):
            li += 1
            ll += sum(pend)
            for k in range(lanes_n):
                if pend[k]:
                    q[k] -= 1
        for k in range(lanes_n):
            if cur[k] is not None and ptr[k] >= len(cur[k]) and q[k] == 0:
                cur[k] = None
        idle = sum(c is None for c in cur)
        busy = lanes_n - idle
        if idle >= R or busy == 0:
            refill()
    return np.array([ni, nl, li, ll], float)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--tiles", type=int, default=24)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--K", default="8,16,32,48")
    a = ap.parse_args()
    W, H = 1920, 1080
    sc = rtamd.Scene(a.scene, W, H, seed=1)
    osc = pyoracle.OracleScene(sc, max_depth=5, spp=4096)
    L = pyoracle.lib()
    L.oracle_trace_log.restype = ctypes.c_long
    L.oracle_trace_log.argtypes = [ctypes.POINTER(pyoracle.OracleSceneDesc)] + [ctypes.c_int] * 8 + [
        ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int32), ctypes.c_long]
    rng = np.random.default_rng(0)
    rf = rtamd.frame_rand_factors(1, 0, a.frames)
    Ks = [int(k) for k in a.K.split(",")]
    A = np.zeros(6)
    B = {k: np.zeros(6) for k in Ks}
    SQ = [(k, qd, st) for k in (64, 32) for qd in (1, 2, 3) for st in ("all",)]
    FR = [(r, qd) for r in (1, 8, 16, 32) for qd in (1, 2, 3)]
    pool = []
    S = {c: np.zeros(6) for c in SQ}
    for _ in range(a.tiles):
        tx, ty = int(rng.integers(0, W // 8)), int(rng.integers(0, H // 8))
        args = (ctypes.byref(osc.desc), W, H, tx * 8, tx * 8 + 8, ty * 8, ty * 8 + 8, 1, a.frames,
                rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        n = L.oracle_trace_log(*args, None, 0)
        buf = np.empty(n, dtype=np.int32)
        L.oracle_trace_log(*args, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n)
        lanes = list(lane_traces(buf).values())
        A += schedule_a(lanes)
        for k in Ks:
            B[k] += schedule_b(lanes, k)
        for c in SQ:
            S[c] += schedule_s(lanes, *c)
        for lt in lanes:
            pool.extend(lt)
    ni, nl, li, ll, si, sl = A
    # calibrate per-iteration costs on A: node 48 %, leaf 35 %, shade 12.6 % of cycles
    cn = 0.419 / ni
    cl = 0.39 / li
    cs = 0.143 / si
    base = ni * cn + li * cl + si * cs
    print(f"scene {a.scene}, {a.tiles} tiles x {a.frames} frames")
    print(f"A: node it {ni:.0f} util {nl / ni / 64:.2f} | leaf it {li:.0f} util {ll / li / 64:.2f} | "
          f"shade it {si:.0f} util {sl / si / 64:.2f} | cost ratios leaf/node {cl / cn:.1f} shade/node {cs / cn:.1f}")
    for k in Ks:
        ni2, nl2, li2, ll2, si2, sl2 = B[k]
        cost = ni2 * cn + li2 * cl + si2 * cs
        print(f"B K={k:2d}: node it {ni2:.0f} util {nl2 / ni2 / 64:.2f} | leaf it {li2:.0f} util {ll2 / li2 / 64:.2f} | "
              f"shade it {si2:.0f} util {sl2 / si2 / 64:.2f} | predicted time {cost / base:.3f} x A")

    rng2 = np.random.default_rng(1)
    order = rng2.permutation(len(pool))
    pool = [pool[k] for k in order]
    for r, qd in FR:
        ni2, nl2, li2, ll2 = schedule_fetch(pool, r, qd)
        cost = ni2 * cn + li2 * cl + si * cs   # shading at schedule A's count (a separate shade pass)
        print(f"F R={r:2d} Q={qd}: node it {ni2:.0f} util {nl2 / ni2 / 64:.2f} | leaf it {li2:.0f} util {ll2 / li2 / 64:.2f}"
              f" | trace cost {(ni2 * cn + li2 * cl) / (ni * cn + li * cl):.3f} x A's trace")
    for c in SQ:
        ni2, nl2, li2, ll2, si2, sl2 = S[c]
        cost = ni2 * cn + li2 * cl + si2 * cs
        print(f"S K={c[0]:2d} Q={c[1]} stop={c[2]:4s}: node it {ni2:.0f} util {nl2 / ni2 / 64:.2f} | leaf it {li2:.0f} "
              f"util {ll2 / li2 / 64:.2f} | shade it {si2:.0f} util {sl2 / si2 / 64:.2f} | predicted {cost / base:.3f} x A")


if __name__ == "__main__":
    main()
