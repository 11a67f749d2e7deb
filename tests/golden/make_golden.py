"""Generate the committed golden fixtures (TEST INFRASTRUCTURE).

For every scene (0-9) at a small size: the CPU oracle's RGBA32F render after a
few progressive frames, plus SHA-256 digests of the scene builder's packed
SSBO/texture/camera bytes.  The reference itself cannot run in this pipeline
(SURVEY §8c), so these vectors pin *our* oracle and scene builder against
regressions; they are not reference outputs.
usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import pyoracle  # noqa: E402
import rtamd  # noqa: E402

# scene, width, height, frames, depth, spp uniform, seed
CASES = [(0, 32, 18, 4, 5, 16, 1), (1, 24, 16, 3, 5, 9, 1), (2, 24, 16, 3, 5, 9, 1), (3, 24, 16, 3, 5, 9, 1),
         (4, 24, 16, 3, 5, 9, 1), (5, 24, 16, 3, 5, 9, 1), (6, 24, 24, 4, 5, 16, 1), (7, 24, 24, 4, 5, 16, 1),
         (8, 32, 18, 4, 5, 16, 1), (9, 40, 24, 4, 8, 16, 1)]


def scene_digest(sc):
    h = {}
    for b in range(6):
        h[f"buf{b}"] = hashlib.sha256(sc.buffers[b]).hexdigest()
    for t in sc.textures:
        h[f"tex{t.slot}"] = hashlib.sha256(t.data).hexdigest() + f":{t.format}:{t.width}x{t.height}"
    h["camera"] = hashlib.sha256(sc.camera.tobytes()).hexdigest()
    return h


def main():
    index = {}
    for sid, w, h, frames, depth, spp, seed in CASES:
        sc = rtamd.Scene(sid, w, h, seed=seed)
        osc = pyoracle.OracleScene(sc, max_depth=depth, spp=spp)
        rf = rtamd.frame_rand_factors(seed, 0, frames)
        img = pyoracle.render(osc, rf)
        name = f"scene{sid}.npz"
        np.savez_compressed(os.path.join(HERE, name), image=img, rand_factors=rf)
        index[str(sid)] = {"file": name, "width": w, "height": h, "frames": frames, "depth": depth, "spp": spp,
                           "seed": seed, "info": sc.info, "digest": scene_digest(sc),
                           "mean_rgb": [float(x) for x in np.nanmean(img[..., :3], axis=(0, 1))]}
        print(sid, index[str(sid)]["mean_rgb"])
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
