"""Analysis (test infrastructure, not collected by pytest): how large is the
union of BVH nodes a wave's lanes visit, per bounce, versus what each lane
visits?  Decides between per-lane and wave-uniform traversal.
usage: python tests/analysis/simt_union.py [--scene 8] [--tiles 40]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--tiles", type=int, default=40)
    ap.add_argument("--frames", type=int, default=4)
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
    stats = {}
    for _ in range(a.tiles):
        tx, ty = int(rng.integers(0, W // 8)), int(rng.integers(0, H // 8))
        args = (ctypes.byref(osc.desc), W, H, tx * 8, tx * 8 + 8, ty * 8, ty * 8 + 8, 1, a.frames,
                rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        n = L.oracle_trace_log(*args, None, 0)
        buf = np.empty(n, dtype=np.int32)
        L.oracle_trace_log(*args, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n)
        k = 0
        groups = {}
        while k < n:
            pix, fr, b, m = buf[k:k + 4]
            groups.setdefault((fr, b), []).append(buf[k + 4:k + 4 + m])
            k += 4 + m
        for (fr, b), seqs in groups.items():
            seqs = [x & 0x3FFFFFFF for x in seqs]
            u = len(set(np.concatenate(seqs).tolist()))
            s = sum(len(x) for x in seqs)
            mx = max(len(x) for x in seqs)
            st = stats.setdefault(b, [0, 0, 0, 0, 0])
            st[0] += 1; st[1] += u; st[2] += s; st[3] += mx; st[4] += len(seqs)
    print(f"scene {a.scene}: per (tile 8x8, frame, bounce)")
    for b in sorted(stats):
        g, u, s, mx, lanes = stats[b]
        print(f" bounce {b}: groups {g} lanes/group {lanes / g:5.1f}  union {u / g:7.1f}  max {mx / g:6.1f}  "
              f"mean/lane {s / lanes:6.1f}  util(uniform)={s / (u * 64.0):5.2f} of 64 lanes; sum/union={s / u:5.1f}")


if __name__ == "__main__":
    main()
