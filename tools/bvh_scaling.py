"""Per-sample cost of BVHs beyond the round-2 link-format cap.

A cloud of N spheres (+ 8 boxes, tests/adversarial.py sphere_cloud) at 1920x1080, max_depth 5,
64 frames per launch, timed with rt_last_render_ns (device time of the launch incl. the
colour fold).  For the ~4000-node cloud, which fits LDS (one 1024-thread workgroup per CU),
the same scene is also rendered with only part of its nodes staged (RT_OPTION_LDS_NODE_CAP:
the two-level walk reads the rest from global memory), so the cost of the two-level walk is
measured on identical work; the ~9800-node cloud needs it by default.
usage: python tools/bvh_scaling.py [--sizes 4000,9000] [--caps 130048,32768] [--extra '{"tl_small_lds": 0}']
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import rtamd  # noqa: E402
import adversarial  # noqa: E402

W, H, FRAMES, DEPTH = 1920, 1080, 64, 5


def timed(scene, options, reps=3):
    ctx = rtamd.RenderContext(devices=(0,), options=options)
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=DEPTH, spp=4096)
    ctx.resize(W, H)
    rf = rtamd.frame_rand_factors(1, 0, FRAMES * (reps + 1))
    ctx.render(1, rf[:FRAMES])   # warm-up
    ctx.sync()
    best = None
    for r in range(reps):
        ctx.render(1 + FRAMES * (r + 1), rf[FRAMES * (r + 1):FRAMES * (r + 2)])
        ns = ctx.last_render_ns()
        best = ns if best is None else min(best, ns)
    info = ctx.last_launch()
    ctx.close()
    return W * H * FRAMES / (best * 1e-9) / 1e6, best * 1e-6, info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-tll0", action="store_true", help="skip the rows with the leaf records in global memory")
    ap.add_argument("--sizes", default="2000,4000,9000")
    ap.add_argument("--extra", default="{}", help="JSON options added to every row's context (e.g. '{\"tl_small_lds\": 0}')")
    ap.add_argument("--caps", default="98304,65536,32768,8192", help="forced LDS node caps (bytes) for the 4000 cloud")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    extra = json.loads(args.extra)
    rows = []
    for n, seed in ((2000, 2), (4000, 4), (9000, 9)):
        if n not in sizes:
            continue
        sc = adversarial.sphere_cloud(n, seed, W=W, H=H)
        caps = [0] if n != 4000 else [0] + [int(c) for c in args.caps.split(",")]
        for cap in caps:
            two_level = bool(cap) or n == 9000
            # the two-level walk with its leaf records in LDS (default) and in global memory
            for tll in ((1, 0) if two_level and not args.no_tll0 else (1,)):
                opts = {"lds_node_cap": cap} if cap else {}
                opts.update(extra)
                if not tll:
                    opts["tl_leaf_lds"] = 0
                rate, ms, info = timed(sc, opts)
                row = {"spheres": n, "bvh_nodes": sc.info["n_bvh_nodes"], "lds_node_cap": cap, "tl_leaf_lds": tll,
                       "Msamples_s": round(rate, 1), "ms_per_launch": round(ms, 3), "shape": info["shape_name"],
                       "block": info["block"], "lds_nodes": info["lds_nodes"], "lds_bytes": info["lds_bytes"],
                       "extra": extra}
                rows.append(row)
                print(json.dumps(row), flush=True)
    if 4000 in sizes:
        base = next(r for r in rows if r["spheres"] == 4000 and r["lds_node_cap"] == 0)["Msamples_s"]
        for r in rows:
            if r["spheres"] == 4000:
                print(json.dumps({"spheres": 4000, "lds_node_cap": r["lds_node_cap"], "tl_leaf_lds": r["tl_leaf_lds"],
                                  "extra": extra, "cost_vs_all_in_lds": round(base / r["Msamples_s"], 3)}),
                      flush=True)


if __name__ == "__main__":
    main()
