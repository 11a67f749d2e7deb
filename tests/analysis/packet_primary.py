"""Analysis (test infrastructure, not collected by pytest): the camera rays of a
group of consecutive pixels of one frame walked as one packet (every lane steps
through the union of the group's node sequences, in the reference's order) —
how many packet steps and packet leaf visits per lane's own steps and leaves?
Groups of 64 (an 8x8 tile), 32 and 16 pixels; bounce 0 only.
usage: python tests/analysis/packet_primary.py [--scene 8] [--tiles 30]"""
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
    ap.add_argument("--tiles", type=int, default=30)
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
    acc = {g: np.zeros(5) for g in (64, 32, 16)}
    for _ in range(a.tiles):
        tx, ty = int(rng.integers(0, W // 8)), int(rng.integers(0, H // 8))
        args = (ctypes.byref(osc.desc), W, H, tx * 8, tx * 8 + 8, ty * 8, ty * 8 + 8, 1, a.frames,
                rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        n = L.oracle_trace_log(*args, None, 0)
        buf = np.empty(n, dtype=np.int32)
        L.oracle_trace_log(*args, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n)
        k = 0
        prim = {}   # frame -> [(pixel, seq)]
        while k < n:
            pix, fr, b, m = buf[k:k + 4]
            if b == 0:
                prim.setdefault(int(fr), []).append((int(pix), buf[k + 4:k + 4 + m].copy()))
            k += 4 + m
        for fr, lst in prim.items():
            lst.sort(key=lambda t: t[0])
            seqs = [s for _, s in lst]
            for g in (64, 32, 16):
                for i in range(0, len(seqs), g):
                    grp = seqs[i:i + g]
                    nodes = set()
                    leaves = set()
                    own_steps = own_leaves = 0
                    for s in grp:
                        nodes.update((s & 0x3FFFFFFF).tolist())
                        lv = s[(s & 0x40000000) != 0] & 0x3FFFFFFF
                        leaves.update(lv.tolist())
                        own_steps += len(s)
                        own_leaves += len(lv)
                    acc[g] += (1, len(nodes), len(leaves), own_steps / len(grp), own_leaves / len(grp))
    print(f"scene {a.scene}: camera rays, packets of consecutive pixels of one frame")
    for g, (cnt, u, ul, st, lv) in acc.items():
        print(f"  group {g:2d}: packet node steps {u / cnt:6.1f} (lane mean {st / cnt:5.1f}, util {st / u:4.2f})  "
              f"packet leaves {ul / cnt:5.2f} (lane mean {lv / cnt:4.2f}, util {lv / ul:4.2f})")


if __name__ == "__main__":
    main()
