#!/usr/bin/env python3
"""Scene 8's gallery residual: does either remaining candidate move the
earth (+4.1..5.6%) and metal (-4.4..6.0%) region offsets against book2_final(scene8).png?

CPU only, oracle probe builds (oracle/Makefile `probe`; the product and the shipped oracle are
unchanged):
  * shipped  -- the oracle as tested (no registered light => the mixture's light
                branch returns vec3(0); rand()'s sin is rt_glsl.h g_sin);
  * sin_f64  -- rand()'s hash with (float)sin((double)x), a correctly rounded sine, instead of the
                shipped polynomial (the reference's vendor sin is NVIDIA's, unknowable here): does
                the hash's stratification quality move the regions?
  * q1_keep  -- Q1 read as "the direction is left unchanged" when there is no light;
  * q1_fog   -- Q1 unchanged for Lambertian surfaces, but an isotropic (fog) scatter keeps its
                direction (the fog is everywhere in scene 8: every path crosses it).
Each renders scene 8 at W x H, depth 6 (the gallery's, profiles/r02_gallery_depth_probe.log),
N spp with the same frames; the regions' linear means (raw floats clipped to [0, 1]) over the
gallery's.  usage: python tools/scene8_residual_probe.py [W H spp] > profiles/r05_scene8_residual_probe.log
       python tools/scene8_residual_probe.py --r6 [W H spp] > profiles/r06_scene8_residual_probe.log
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "raytracing-book_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import gallery_regions as gr  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

FIX = json.load(open(os.path.join(REPO, "tests", "golden", "gallery.json")))
REGIONS = ("glass", "metal", "blue_fog", "earth", "perlin")
BUILD = os.path.join(REPO, "oracle", "build")
VARIANTS = [("shipped", "liboracle.so", 6), ("sin_f64", "liboracle_probe_sin.so", 6),
            ("q1_keep", "liboracle_probe_q1a.so", 6), ("q1_fog", "liboracle_probe_q1b.so", 6)]
# round 6 (--r6): the gallery's depth on the metal region alone, and the metal
# scatter's fuzz forms -- reflect(unit(dir)) + fuzz * random_in_unit_sphere (the book's earlier
# form), and the reflected direction left unnormalised
VARIANTS_R6 = [("shipped", "liboracle.so", 6), ("depth5", "liboracle.so", 5),
               ("metal_ball", "liboracle_probe_metal1.so", 6), ("metal_raw", "liboracle_probe_metal2.so", 6)]


def main():
    r6 = "--r6" in sys.argv
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    W, H, spp = (int(x) for x in (args[:3] if len(args) > 2 else (400, 300, 256)))
    os.system(f"make -s -C {os.path.join(REPO, 'oracle')} all probe")
    sc = rtamd.Scene(8, W, H, seed=1)
    regs = gr.scene8_regions(sc.camera, W, H, erode=1)
    fx = FIX["scene8_regions"]["regions"]
    rf = rtamd.frame_rand_factors(1, 0, spp)
    print(f"scene 8, {W}x{H}, {spp} spp, depth 6, seed 1: linear region mean (raw floats clipped to [0, 1]) / "
          f"gallery's linearised mean, per channel; px per region: "
          f"{ {n: int(regs[n].sum()) for n in REGIONS} }", flush=True)
    base = None
    for name, lib, depth in (VARIANTS_R6 if r6 else VARIANTS):
        pyoracle.LIB, pyoracle._L = os.path.join(BUILD, lib), None
        t = time.time()
        img = pyoracle.render(pyoracle.OracleScene(sc, max_depth=depth, spp=spp), rf, nthreads=os.cpu_count())
        lin = np.clip(np.nan_to_num(img[..., :3].astype(np.float64), nan=0.0), 0.0, 1.0)
        ratio = {n: lin[regs[n]].mean(0) / np.array(fx[n]["lin_mean"]) for n in REGIONS}
        if base is None:
            base = ratio
        rel = {n: ratio[n] / base[n] for n in REGIONS}
        print(f"{name:8s} ({time.time() - t:5.1f} s) " +
              "  ".join(f"{n} {np.round(ratio[n], 3).tolist()}" for n in REGIONS), flush=True)
        if name != "shipped":
            print(f"{'':8s}   vs shipped: " + "  ".join(f"{n} {np.round(rel[n], 3).tolist()}" for n in REGIONS),
                  flush=True)
    pyoracle.LIB, pyoracle._L = os.path.join(BUILD, "liboracle.so"), None


if __name__ == "__main__":
    main()
