"""Leaf census (VERDICT r5 Next 1): could a workgroup-wide leaf-task queue per prim type fill lanes?

Runs the stats twin (A/B library) with the census on (rt_debug_enable_stats(ctx, 2)): every wave
leaf round leaves one record -- when it started and how long it took (s_memtime cycles), its
workgroup and wave, how many lanes were walking, and per prim type how many lanes hold a slot-0 and
a slot-1 test.  Then, per workgroup (one per CU on scene 8: 16 waves sharing the LDS a queue would
live in):

* today: lanes per wave execution of each type's block (one execution per wave round with >= 1
  such lane; the stats twin's `lanes/exec`);
* pooled by window: the rounds that START in the same W-cycle window of one workgroup pooled per
  type and slot into ceil(n / 64) executions -- the lanes per execution a queue could reach if it
  gathered a window's tasks (W from a fraction of a leaf round to several);
* pooled by overlap: at the start of each round, the lanes of that type in every round of the
  workgroup in progress at that moment (the tasks a queue would hold at once), as a distribution.

usage: python tools/leaf_census.py [--scene 8] [--frames 4] [--save gpurun_out/census.npz]
       python tools/leaf_census.py --load profiles/r06_leaf_census_s8.npz   (analysis only, CPU)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TYPES = ["SPH", "QUAD", "MED", "BOX"]   # RT_MODEL_SPHERE = 1, QUAD = 2, CONSTANT_MEDIUM = 3, BOX = 4


def collect(a):
    sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
    import rtamd
    scene = rtamd.Scene(a.scene, a.width, a.height, seed=1)
    ctx = rtamd.RenderContext(devices=(0,), ab=True)
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=a.depth, spp=4096)
    ctx.resize(a.width, a.height)
    L = rtamd.amd_ab()
    assert L.rt_debug_enable_stats(ctx._h, 2) == 0
    ctx.render(1, rtamd.frame_rand_factors(1, 0, a.frames))
    ctx.sync()
    need, waves, cap = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_int()
    assert L.rt_debug_read_census(ctx._h, None, 0, ctypes.byref(need), ctypes.byref(waves), ctypes.byref(cap)) == 0
    buf = np.zeros(need.value, dtype=np.uint32)
    assert L.rt_debug_read_census(ctx._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint)), need.value, None,
                                  None, None) == 0
    stats = (ctypes.c_ulonglong * 128)()
    assert L.rt_debug_read_stats(ctx._h, stats, 128) == 0
    info = ctx.last_launch() if hasattr(ctx, "last_launch") else None
    ctx.close()
    nw, cp = waves.value, cap.value
    counts = buf[:nw].astype(np.int64)
    recs = buf[nw:].reshape(nw, cp, 5)
    clipped = int((counts > cp).sum())
    rows = [recs[w, :min(int(counts[w]), cp)] for w in range(nw) if counts[w] > 0]
    ev = np.concatenate(rows) if rows else np.zeros((0, 5), np.uint32)
    meta = {"scene": a.scene, "width": a.width, "height": a.height, "frames": a.frames, "depth": a.depth,
            "waves": nw, "cap": cp, "waves_clipped": clipped, "records": int(ev.shape[0]),
            "records_lost": int(np.maximum(counts - cp, 0).sum())}
    return ev, meta


def unpack(ev):
    t0 = ev[:, 0].astype(np.int64)
    dur = ev[:, 1].astype(np.int64)
    wg = (ev[:, 2] & 0xFFFF).astype(np.int64)
    wave = ((ev[:, 2] >> 16) & 0xFF).astype(np.int64)
    walking = ((ev[:, 2] >> 24) & 0xFF).astype(np.int64)
    s0 = np.stack([(ev[:, 3] >> (8 * k)) & 0xFF for k in range(4)], 1).astype(np.int64)
    s1 = np.stack([(ev[:, 4] >> (8 * k)) & 0xFF for k in range(4)], 1).astype(np.int64)
    # s_memtime wraps at 2^32 in the record: unwrap per workgroup around its first record
    return t0, dur, wg, wave, walking, s0, s1


def analyse(ev, meta, out):
    p = out.append
    t0, dur, wg, wave, walking, s0, s1 = unpack(ev)
    n = len(t0)
    p("# leaf census: scene %(scene)d %(width)dx%(height)d x %(frames)d frames, depth %(depth)d" % meta)
    p("records %d (lost to the per-wave cap: %d; waves clipped %d of %d)" % (n, meta["records_lost"],
                                                                          meta["waves_clipped"], meta["waves"]))
    wgs = np.unique(wg)
    p("workgroups %d, waves per workgroup seen %d; wave leaf rounds per workgroup %.0f" %
      (len(wgs), int(wave.max()) + 1, n / max(len(wgs), 1)))
    p("leaf round: cycles p10 / p50 / p90 = %d / %d / %d; walking lanes mean %.1f" %
      (np.percentile(dur, 10), np.percentile(dur, 50), np.percentile(dur, 90), walking.mean()))
    # today
    p("")
    p("today (one execution per wave round with >= 1 lane of the type):")
    today = {}
    for k, tn in enumerate(TYPES):
        for s, arr in ((0, s0), (1, s1)):
            c = arr[:, k]
            ex = int((c > 0).sum())
            if ex == 0:
                continue
            today[(tn, s)] = (int(c.sum()), ex)
            p("  %-4s slot %d: executions %9d, lanes %10d, lanes/exec %5.2f" % (tn, s, ex, c.sum(), c.sum() / ex))
    # the record keeps s_memtime's low 32 bits (1.8 s at 2.4 GHz, far more than a launch): per
    # workgroup, unwrap a wrap inside the launch, then times relative to its first record
    tt = t0.copy()
    for g in wgs:
        m = wg == g
        x = t0[m].copy()
        if x.max() - x.min() > (1 << 31):
            x[x < (1 << 31)] += 1 << 32
        tt[m] = x - x.min()
    order = np.lexsort((tt, wg))
    tt, dur, wg, wave, s0, s1 = tt[order], dur[order], wg[order], wave[order], s0[order], s1[order]
    p("")
    p("pooled by window (the rounds of one workgroup starting in the same W-cycle window; per type and slot,")
    p("ceil(lanes / 64) executions): lanes per execution, and executions relative to today")
    med = int(np.percentile(dur, 50))
    windows = sorted(set([250, 500, 1000, 2000, 4000, 8000, 16000, med]))
    p("  %-10s" % "W cycles" + "".join("%16s" % ("%s s%d" % key) for key in today))
    res = {}
    for W in windows:
        b = wg * (1 << 40) + tt // W
        ub, inv = np.unique(b, return_inverse=True)
        row = []
        for key, (lanes, ex) in today.items():
            k = TYPES.index(key[0])
            c = (s0 if key[1] == 0 else s1)[:, k]
            tot = np.bincount(inv, weights=c, minlength=len(ub))
            pe = int(np.ceil(tot / 64.0).sum())
            res[(W, key)] = (lanes / max(pe, 1), pe / ex)
            row.append("%7.2f (%4.2fx)" % (lanes / max(pe, 1), pe / ex))
        p("  %-10s" % ("%d%s" % (W, " (p50)" if W == med else "")) + "".join("%16s" % r for r in row))
    # pooled by overlap: at each round's start, the lanes of the type in every round of its
    # workgroup in progress then (itself included)
    p("")
    p("pooled by overlap (tasks a workgroup queue would hold at once): at each round's start, the lanes of")
    p("the type in all rounds of the workgroup then in progress; percentiles over rounds with >= 1 such lane")
    p("  %-10s %8s %8s %8s %8s %8s   %s" % ("type/slot", "p10", "p25", "p50", "p75", "p90", "rounds in progress p50"))
    for key in today:
        k = TYPES.index(key[0])
        c = (s0 if key[1] == 0 else s1)[:, k]
        pooled, conc = [], []
        for g in wgs:
            m = np.nonzero(wg == g)[0]
            st, en, cc = tt[m], tt[m] + dur[m], c[m]
            # starts sorted (lexsort above); rounds in progress at st[i]: started at or before, ending after
            cs = np.concatenate([[0], np.cumsum(cc)])
            ends_sorted = np.sort(en)
            idx_start = np.searchsorted(st, st, side="right")          # rounds started <= st[i]
            # lanes of rounds started <= st[i] minus those of rounds that ended <= st[i]
            e_order = np.argsort(en)
            ce = np.concatenate([[0], np.cumsum(cc[e_order])])
            idx_end = np.searchsorted(ends_sorted, st, side="right")
            lanes_now = cs[idx_start] - ce[idx_end]
            n_now = idx_start - idx_end
            sel = cc > 0
            pooled.append(lanes_now[sel])
            conc.append(n_now[sel])
        pl = np.concatenate(pooled)
        cn = np.concatenate(conc)
        q = np.percentile(pl, [10, 25, 50, 75, 90])
        p("  %-10s %8.1f %8.1f %8.1f %8.1f %8.1f   %.0f" % ("%s s%d" % key, *q, np.percentile(cn, 50)))
        res[("overlap", key)] = [float(x) for x in q]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--save", default=None, help="npz of the records and meta")
    ap.add_argument("--load", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.load:
        z = np.load(a.load)
        ev, meta = z["ev"], json.loads(str(z["meta"]))
    else:
        ev, meta = collect(a)
        if a.save:
            np.savez_compressed(a.save, ev=ev, meta=json.dumps(meta))
    out = []
    analyse(ev, meta, out)
    txt = "\n".join(out)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
