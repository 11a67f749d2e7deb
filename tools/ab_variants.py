"""Interleaved in-process A/B of kernel structure variants (RT_KERNEL_VARIANT).

Every variant must produce the same bits; timings are HIP-event device time of
one rt_render call (1 launch) per round, reported as median/min over rounds.
A variant spec is "<RT_KERNEL_VARIANT>" optionally followed by c<RT_CHUNK_TARGET>,
k<RT_SHADE_K>, d<RT_DEBUG_FLAGS> (ablations: bits differ by design) and/or
s<RT_STAGE_TILES>, b<RT_SM_BATCH>, f<RT_SM_FRAC>, x<RT_FASTDIV>, w<RT_WALK_FRAC>, p<RT_BOX_PRETEST>, t<RT_STAGED_CHUNK_TARGET>, h<RT_SPH_LDS>, g<RT_BIG_WG> (e.g. 30c0 = variant 30 with one unit per tile; 0s0 = ordered
chunks whatever the tile count; 0s1000 = staged chunks).
usage: python tools/ab_variants.py [--variants 30c0,30c16] [--rounds 5] [--scene 8]
"""
import argparse
import os

os.environ.setdefault("RTAMD_LIB", "ab")   # the A/B build reads the RT_* knobs (rtamd._lib.amd)
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
import numpy as np  # noqa: E402
import rtamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="30c0,30c16")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--stripe-rows", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--depth", type=int, default=5)
    a = ap.parse_args()
    variants = a.variants.split(",")
    scene = rtamd.Scene(a.scene, a.width, a.height, seed=1)
    ctxs = {}
    for v in variants:
        import re
        m = re.fullmatch(r"(\d+)(?:c(\d+))?(?:k(\d+))?(?:d(\d+))?(?:s(\d+))?(?:b(\d+))?(?:f(\d+))?(?:x(\d+))?(?:w(\d+))?(?:p(\d+))?(?:t(\d+))?(?:h(\d+))?(?:g(\d+))?", v)
        assert m, f"bad variant spec {v}"
        os.environ["RT_KERNEL_VARIANT"] = m.group(1)
        for env, val in (("RT_CHUNK_TARGET", m.group(2)), ("RT_SHADE_K", m.group(3)), ("RT_DEBUG_FLAGS", m.group(4)),
                         ("RT_STAGE_TILES", m.group(5)), ("RT_SM_BATCH", m.group(6)),
                         ("RT_SM_FRAC", m.group(7)), ("RT_FASTDIV", m.group(8)),
                         ("RT_WALK_FRAC", m.group(9)), ("RT_BOX_PRETEST", m.group(10)),
                         ("RT_STAGED_CHUNK_TARGET", m.group(11)), ("RT_SPH_LDS", m.group(12)), ("RT_BIG_WG", m.group(13))):
            if val:
                os.environ[env] = val
            else:
                os.environ.pop(env, None)
        c = rtamd.RenderContext(devices=(0,), rank=a.rank, world=a.world, stripe_rows=a.stripe_rows)
        c.upload_scene(scene)
        c.set_params(max_depth=a.depth, spp=4096)
        c.resize(a.width, a.height)
        ctxs[v] = c
    rf = rtamd.frame_rand_factors(1, 0, a.frames)
    times = {v: [] for v in variants}
    ref = None
    for r in range(a.rounds + 1):
        for v in variants:
            c = ctxs[v]
            c.resize(a.width, a.height)      # zero the image: same inputs every round
            c.render(1, rf)
            c.sync()
            ns = c.last_render_ns()
            if r == 0:   # warm-up round; check bits
                img = c.read_image()
                if ref is None:
                    ref = img
                else:
                    same = np.array_equal(np.isnan(img), np.isnan(ref)) and np.array_equal(
                        img.view(np.uint32)[~np.isnan(img)], ref.view(np.uint32)[~np.isnan(ref)])
                    print(f"variant {v}: bits {'identical' if same else 'DIFFER'} to variant {variants[0]}")
                continue
            times[v].append(ns / 1e6)
    samples = a.width * rtamd.local_rows(a.height, a.rank, a.world, a.stripe_rows) * a.frames
    for v in variants:
        med = statistics.median(times[v])
        print(f"variant {v}: median {med:.2f} ms  min {min(times[v]):.2f} ms  -> {samples / med / 1e3:.1f} Msamples/s")


if __name__ == "__main__":
    main()
