"""Region means of scene 8 (800x600, 4096 spp, HIP kernel) against the reference's gallery
image at several max_depth values: which depth the published render most likely used
(the reference records none; the GUI slider spans 1-50, the CLI default is 5)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import rtamd  # noqa: E402
import gallery_regions as gr  # noqa: E402

FIX = json.load(open(os.path.join(REPO, "tests", "golden", "gallery.json")))


def main():
    sc = rtamd.Scene(8, 800, 600, seed=1)
    regs = gr.scene8_regions(sc.camera, 800, 600)
    fx = FIX["scene8_regions"]["regions"]
    rf = rtamd.frame_rand_factors(1, 0, 4096)
    for depth in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "5,8,10,20,50").split(",")]:
        ctx = rtamd.RenderContext(devices=(0,))
        ctx.upload_scene(sc)
        ctx.set_params(max_depth=depth, spp=4096)
        ctx.resize(800, 600)
        for k in range(0, 4096, 512):
            ctx.render(k + 1, rf[k:k + 512])
        img = ctx.read_image()
        ctx.close()
        lin = np.clip(np.nan_to_num(img[..., :3], nan=0.0), 0.0, 1.0)
        rep = {n: np.round(lin[regs[n]].mean(0) / np.array(fx[n]["lin_mean"]), 3).tolist()
               for n in ("glass", "metal", "blue_fog", "earth", "perlin")}
        worst = max(abs(x - 1.0) for v in rep.values() for x in v)
        print(json.dumps({"max_depth": depth, "worst_rel_dev": round(worst, 3), "ratios": rep}), flush=True)


if __name__ == "__main__":
    main()
