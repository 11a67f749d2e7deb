"""Run the diagnostic stats build of the render kernel and print where wave time
goes (s_memtime per region, once per wave) and each region's SIMD lane use.
usage: python tools/kernel_stats.py [--scene 8] [--frames 16] [--width 1920 --height 1080] [--options JSON]"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
import rtamd  # noqa: E402

NAMES = ["TOTAL", "START_CYC", "START_IT", "START_LN", "NODE_CYC", "NODE_IT", "NODE_LN", "LEAF_CYC", "LEAF_IT",
         "LEAF_LN", "SPH_LN", "QUAD_LN", "BOX_LN", "MED_LN", "SHADE_CYC", "SHADE_IT", "SHADE_LN", "SPH_IT",
         "QUAD_IT", "BOX_IT", "MED_IT", "FAST_TRACES", "FAST_EXACT"] + [f"FAST_WHY{r}" for r in range(1, 10)] + [
         "FAST_STEPS", "FAST_TESTS", "FAST_PRE_CYC", "FAST_POST_CYC", "FAST_EXACT_CYC",
         "SPH_CYC", "QUAD_CYC", "BOX_CYC", "MED_CYC", "TRACE_IT", "TRACE_LN", "ROUND_IT", "ROUND_LN",
         "RET_IT", "RET_LN", "SPH_SM", "QUAD_SM", "BOX_SM", "MED_SM", "NODE_SM",
         "SH_HIT_CYC", "SH_SCAT_CYC", "SH_MIX_CYC", "SH_TEX_CYC", "SH_LAM_IT", "SH_LAM_LN", "SH_ISO_IT", "SH_ISO_LN",
         "SH_MET_IT", "SH_MET_LN", "SH_DIE_IT", "SH_DIE_LN",
         "PASS_IT", "PASS_CYC", "WATCH_CYC", "FOLD_CYC", "CLAIM_CYC", "CLAIM_IT", "UNIT_IT", "ATOM_CYC",
         "BEGIN_CYC", "ROUNDS_CYC", "RHEAD_CYC", "SHBLK_CYC", "PTAIL_CYC", "CEN_N"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--options", default="{}", help='JSON, e.g. {"leaf_defer": 16}')
    ap.add_argument("--cloud", type=int, default=0, help="N > 0: tests/adversarial.py sphere_cloud(N) instead of --scene")
    a = ap.parse_args()
    import json
    if a.cloud:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import adversarial
        seeds = {2000: 2, 4000: 4, 9000: 9}
        scene = adversarial.sphere_cloud(a.cloud, seeds.get(a.cloud, 1), W=a.width, H=a.height)
    else:
        scene = rtamd.Scene(a.scene, a.width, a.height, seed=1)
    ctx = rtamd.RenderContext(devices=(0,), ab=True, options=json.loads(a.options) or None)   # the stats kernels are in the A/B build
    ctx.upload_scene(scene)
    ctx.set_params(max_depth=a.depth, spp=4096)
    ctx.resize(a.width, a.height)
    L = rtamd.amd_ab()
    assert L.rt_debug_enable_stats(ctx._h, 1) == 0
    ctx.render(1, rtamd.frame_rand_factors(1, 0, a.frames))
    ctx.sync()
    buf = (ctypes.c_ulonglong * 128)()
    assert L.rt_debug_read_stats(ctx._h, buf, 128) == 0
    v = {n: buf[i] for i, n in enumerate(NAMES)}
    tot = v["TOTAL"] or 1
    samples = a.width * a.height * a.frames
    print(f"{'cloud ' + str(a.cloud) if a.cloud else 'scene ' + str(a.scene)} {json.loads(a.options)} {a.width}x{a.height}x{a.frames}: {samples} samples, wave-cycles total {tot:.3e}")
    for reg in ["START", "NODE", "LEAF", "SHADE"]:
        cyc, it, ln = v[reg + "_CYC"], v[reg + "_IT"], v[reg + "_LN"]
        util = ln / (64.0 * it) if it else 0
        print(f"  {reg:6s} {100.0 * cyc / tot:5.1f}% of wave-cycles  iterations {it:.3e}  lane-util {100 * util:5.1f}%  "
              f"cyc/iter {cyc / max(it, 1):7.1f}  lane-iters/sample {ln / samples:6.2f}")
    for t in ["SPH", "QUAD", "BOX", "MED"]:
        it, ln = v[t + "_IT"], v[t + "_LN"]
        cyc = v[t + "_CYC"]
        print(f"  leaf-slot {t:4s}: wave-executions {it:.3e} lanes/exec {ln / max(it, 1):5.2f}  per-sample {ln / samples:5.2f}"
              f"  {100.0 * cyc / tot:5.1f}% of wave-cycles  cyc/exec {cyc / max(it, 1):7.1f}")
    if v["TRACE_IT"]:
        print(f"  link walk: {v['TRACE_LN'] / v['TRACE_IT']:5.2f} lanes per wave trace, "
              f"{v['ROUND_IT'] / v['TRACE_IT']:5.2f} node-walk+leaf rounds per wave trace, "
              f"{v['ROUND_LN'] / (64.0 * max(v['ROUND_IT'], 1)) * 100:5.1f}% of lanes still tracing per round")
    if v["SH_HIT_CYC"]:
        print("  shading parts: " + "  ".join(f"{k} {100.0 * v['SH_' + k + '_CYC'] / tot:4.1f}%" for k in ("HIT", "SCAT", "MIX", "TEX"))
              + " of wave-cycles")
        for m in ("LAM", "ISO", "MET", "DIE"):
            it, ln = v[f"SH_{m}_IT"], v[f"SH_{m}_LN"]
            print(f"  material {m}: wave-executions {it:.3e} lanes/exec {ln / max(it, 1):5.2f}  per-sample {ln / samples:5.2f}")
    if v["ROUND_IT"]:
        print(f"  rounds with retired lanes: {v['RET_IT'] / v['ROUND_IT'] * 100:5.1f}% of rounds, "
              f"{v['RET_LN'] / (64.0 * v['ROUND_IT']) * 100:5.1f}% of lane-rounds retired (unit tails)")
    if v["PASS_IT"]:
        # render_stream's passes (round 6): each part's wave-cycles; the claim loop holds START, the
        # rounds hold NODE and LEAF, the shading block holds SHADE (its first-lane timer)
        pc = v["PASS_CYC"]
        print(f"  passes {v['PASS_IT']:.3e} ({v['PASS_IT'] / max(v['ROUND_IT'], 1):.2f} per round), "
              f"{100.0 * pc / tot:5.1f}% of wave-cycles inside passes; parts, % of wave-cycles:")
        parts = [("watchdog", v["WATCH_CYC"]), ("unit folds", v["FOLD_CYC"]),
                 ("claim loop - START", v["CLAIM_CYC"] - v["START_CYC"]), ("  of it the unit atomic", v["ATOM_CYC"]),
                 ("new walks' set-up", v["BEGIN_CYC"]),
                 ("rounds - NODE - LEAF", v["ROUNDS_CYC"] - v["NODE_CYC"] - v["LEAF_CYC"]),
                 ("  of it the loop heads", v["RHEAD_CYC"]),
                 ("shading block - SHADE", v["SHBLK_CYC"] - v["SHADE_CYC"]), ("pass tail", v["PTAIL_CYC"]),
                 ("outside passes", tot - pc)]
        for name, c in parts:
            print(f"    {name:24s} {100.0 * c / tot:5.1f}%")
        named = v["START_CYC"] + v["NODE_CYC"] + v["LEAF_CYC"] + v["SHADE_CYC"]
        print(f"  START+NODE+LEAF+SHADE {100.0 * named / tot:5.1f}%; claim-loop iterations {v['CLAIM_IT'] / max(v['PASS_IT'], 1):.2f}"
              f" per pass, units {v['UNIT_IT']:.3e}, unit atomic {v['ATOM_CYC'] / max(v['UNIT_IT'], 1):.0f} cycles each")
    print("raw", v)


if __name__ == "__main__":
    main()
