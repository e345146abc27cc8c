"""Parity probe of one librt4.so build on the all_primitives kernel (builds that differ
only in scheduling or in a pure-predicate rewrite must compute the same images and counts).

Usage (GPU box, one build per process so that a hang ends with its own time limit):
  RT4_LIB=<build .so> python tools/variant_probe.py <label> [scene]
  (RT4_PROBE_SINGLE=1: the two single-frame renders only)

For the 96x60 4 spp 4 bounce frame of test_gpu_parity.py (LUT and inline Newton kernels) and a pipelined
8-frame 128x96 progressive call, prints the count against the oracle's, the number of differing pixels and
how they differ (GPU pixel left at its old value, NaN, other), and the first few coordinates. Exits 0 on a
mismatch (this is a diagnostic); only an exception or a hang (the caller's timeout) stops the chain."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

rt4 = importlib.import_module("4d_ray_tracing_amd")
import oracle_lib  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "tree"
scene_name = sys.argv[2] if len(sys.argv) > 2 else "all_primitives"
scene = rt4.Scene.named(scene_name)


def describe(tag, fg, ng, fc, nc, old):
    diff = np.any(fg != fc, axis=2)
    nd = int(diff.sum())
    stale = int(np.sum(diff & np.all(fg == old, axis=2)))
    nan = int(np.sum(diff & np.any(np.isnan(fg), axis=2)))
    where = np.argwhere(diff)[:6].tolist()
    md = float(np.nanmax(np.abs(fg - fc))) if nd else 0.0
    print(f"{label:>10s} {tag:<18s} count {ng} vs {nc} ({ng - nc:+d})  differing px {nd} (stale {stale}, nan {nan}) "
          f"max|d| {md:.3g}  first {where}", flush=True)


def single(flags, tag):
    u = rt4.make_uniforms(96, 60, samples=4, reflections=4, seed=777)
    reg = rt4.region(96, 60)
    t = rt4.Tracer(device=0, flags=flags, scene=scene)
    old = np.full((60, 96, 4), 0.25, np.float32)
    fg = old.copy()
    ng = t.render_host(u, reg, fg)
    t.close()
    fc, nc, _, _ = oracle_lib.render(scene.desc, u, reg, old.copy())
    describe(tag, fg, ng, fc, nc, old)


def pipelined(flags, tag, w=128, h=96, n=8):
    base = rt4.make_uniforms(w, h, samples=2, reflections=4, seed=4242)
    us = [rt4.progressive_uniforms(base, f + 1) for f in range(n)]
    reg = rt4.region(w, h)
    t = rt4.Tracer(device=0, flags=flags, scene=scene)
    frame = torch.full((h, w, 4), 0.25, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    t.render_frames_device(us, reg, frame.data_ptr(), rt4.FRAME_RGBA32F, w, cnt.data_ptr())
    torch.cuda.synchronize()
    fg, ng = frame.cpu().numpy(), int(cnt.item())
    t.close()
    old = np.full((h, w, 4), 0.25, np.float32)
    fc, nc = old.copy(), 0
    for uf in us:
        fc, k, _, _ = oracle_lib.render(scene.desc, uf, reg, fc)
        nc += k
    describe(tag, fg, ng, fc, nc, old)


single(rt4.FLAG_SAMPLER_LUT, "lut 96x60")
single(0, "inline 96x60")
if os.environ.get("RT4_PROBE_SINGLE") != "1":
    pipelined(rt4.FLAG_SAMPLER_LUT, "lut pipelined x8")
print(f"{label} done", flush=True)
