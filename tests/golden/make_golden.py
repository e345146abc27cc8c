"""Regenerates the golden fixtures of tests/golden from the CPU oracle (test infrastructure).

  images.json + image_<scene>.npy : small renders of the five reference scenes (oracle output), the
                                    GPU's pin in test_gpu_parity.test_golden_images
  sampler.json                    : exhaustive w_by_volume sweep statistics (iteration histogram)

The RNG / sampler known-answer vectors in kat.json are NOT generated here: they are the values
SURVEY.md §4 derived from the reference's shader.frag:94-158 and are kept verbatim.
Run: python tests/golden/make_golden.py
"""
import importlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
rt4 = importlib.import_module("4d_ray_tracing_amd")
import oracle_lib  # noqa: E402

SCENES = ["sphere", "room", "tiger", "cylinder4d", "hypercube"]
W, H, SPP, B, SEED = 48, 30, 3, 3, 20240607


def main():
    meta = {}
    for name in SCENES:
        scene = rt4.Scene.builtin(name)
        u = rt4.make_uniforms(W, H, samples=SPP, reflections=B, seed=SEED)
        f, n, _, _ = oracle_lib.render(scene.desc, u, rt4.region(W, H), threads=4)
        np.save(os.path.join(HERE, f"image_{name}.npy"), f)
        meta[name] = {"width": W, "height": H, "samples": SPP, "reflections": B, "seed": SEED, "intersections": int(n),
                      "mean_rgb": [float(x) for x in f[..., :3].reshape(-1, 3).mean(0)]}
    json.dump(meta, open(os.path.join(HERE, "images.json"), "w"), indent=1)
    v = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)
    w, it = oracle_lib.eval_array(rt4.EVAL_W_BY_VOLUME, v)
    hist = np.bincount(it, minlength=int(it.max()) + 1)
    json.dump({"inputs": int(v.size), "max_iterations": int(it.max()), "mean_iterations": float(it.mean()),
               "histogram": [int(x) for x in hist], "nan": int(np.isnan(w).sum()), "max_abs_w": float(np.abs(w).max())},
              open(os.path.join(HERE, "sampler.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
