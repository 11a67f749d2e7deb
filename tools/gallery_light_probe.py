"""Scene 8 with and without its light quad registered as a light.

Scene.java:301-302 adds scene 8's DiffuseLight quad as a model only (RaytraceModel.addModel,
never addLight), so the reference's ray colour takes its no-light branch
and tests/test_gallery_anchor.py's regions compare against that.  The gallery is less noisy
than a 4096-spp render of that branch (tools/gallery_spp_probe.py); this renders the scene
(built through rtamd.SceneBuilder from Scene.java:282-343, unseeded parts from numpy) both
ways on the GPU at 800x600, max_depth 6, 4096 spp, and reports the regions' mean ratios and
neighbour-difference noise against the gallery, to see whether a render with light sampling
is what the gallery shows.
usage: python tools/gallery_light_probe.py [spp]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import rtamd  # noqa: E402
import gallery_regions as gr  # noqa: E402
from rtamd.scene import SceneBuilder  # noqa: E402

FIX = json.load(open(os.path.join(REPO, "tests", "golden", "gallery.json")))
REGIONS = ("glass", "metal", "blue_fog", "earth", "perlin")


def build(with_light, W=800, H=600, seed=7):
    rng = np.random.default_rng(seed)
    b = SceneBuilder(seed=1)
    ground = b.lambertian(b.solid(0.48, 0.83, 0.53))
    for i in range(20):
        for j in range(20):
            x0, z0 = -1000.0 + i * 100.0, -1000.0 + j * 100.0
            b.add(b.box((x0, 0.0, z0), (x0 + 100.0, float(np.float32(1 + rng.random() * 100)), z0 + 100.0), ground))
    lq = b.add(b.quad((123, 554, 147), (300, 0, 0), (0, 0, 265), b.diffuse_light(7, 7, 7)))
    if with_light:
        b.add_light(lq)
    b.add(b.sphere((400, 400, 200), 50, b.lambertian(b.solid(0.7, 0.3, 0.1)), center2=(500, 400, 200)))
    b.add(b.sphere((260, 150, 45), 50, b.dielectric(1.5)))
    b.add(b.sphere((0, 150, 145), 50, b.metal(b.solid(0.8, 0.8, 0.9), 0.999)))
    bd = b.add(b.sphere((360, 150, 145), 70, b.dielectric(1.5)))
    b.add(b.constant_medium(bd, 0.2, b.isotropic(b.solid(0.2, 0.4, 0.9))))
    bd2 = b.sphere((0, 0, 0), 5000, b.dielectric(1.5))
    b.add(b.constant_medium(bd2, 0.0001, b.isotropic(b.solid(1, 1, 1))))
    b.add(b.sphere((400, 200, 400), 100, b.lambertian(b.image("earthmap.ppm", 100, 0))))
    b.add(b.sphere((220, 280, 300), 80, b.lambertian(b.perlin(0.2))))
    white = b.lambertian(b.solid(0.73, 0.73, 0.73))
    for _ in range(1000):
        c = np.float32(165 * rng.random(3)) + np.float32([-100, 270, 395])
        b.add(b.sphere(tuple(float(v) for v in c), 10, white))
    b.camera(look_from=(478, 278, -600), look_at=(278, 278, 0), vfov=40, background=(0, 0, 0))
    return b.finish(W, H)


def dx2(lin, m):
    both = m[:, 1:] & m[:, :-1]
    d = lin[:, 1:] - lin[:, :-1]
    return (d[both] ** 2).mean(0)


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    fx = FIX["scene8_regions"]["regions"]
    for with_light in (False, True):
        sc = build(with_light)
        ctx = rtamd.RenderContext(devices=(0,))
        ctx.upload_scene(sc)
        ctx.set_params(max_depth=6, spp=spp)
        ctx.resize(800, 600)
        rf = rtamd.frame_rand_factors(1, 0, spp)
        for k in range(0, spp, 512):
            ctx.render(k + 1, rf[k:k + 512])
        img = ctx.read_image()
        ctx.close()
        regs = gr.scene8_regions(sc.camera, 800, 600)
        lin = (rtamd.tonemap_rgb8(img).astype(np.float64) / 255.0) ** 2.2
        rep = {r: {"mean": np.round(lin[regs[r]].mean(0) / np.array(fx[r]["lin_mean"]), 4).tolist(),
                   "dx2": np.round(dx2(lin, regs[r]) / np.array(fx[r]["lin_dx2"]), 4).tolist()} for r in REGIONS}
        print(json.dumps({"light_registered": with_light, "spp": spp, "max_depth": 6, "regions": rep}), flush=True)


if __name__ == "__main__":
    main()
