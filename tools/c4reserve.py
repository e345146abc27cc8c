#!/usr/bin/env python3
"""Config-4 frame-by-frame timing with and without a 4 GiB frame-colour reservation in the same context
(does the large allocation slow the spilling mirror-room kernel?). Usage: python tools/c4reserve.py"""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

rt4 = importlib.import_module("4d_ray_tracing_amd")
scene = rt4.Scene.named(sys.argv[1] if len(sys.argv) > 1 else "tiger_two_mirrors")
w, h = 3840, 2160
u = rt4.make_uniforms(w, h, samples=int(sys.argv[2]) if len(sys.argv) > 2 else 16, reflections=12, seed=12345)
reg = rt4.region(w, h)
for reserve in (False, True, False):
    t = rt4.Tracer(0, rt4.FLAG_SAMPLER_LUT, scene)
    if reserve:
        t.reserve_frames(4000, 2100)  # 32 x 4000 x 2100 x 16 B, a size the 4K frame never asks for
    fr = torch.zeros((h, w, 4), device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    t.render_device(u, reg, fr.data_ptr(), w, 0, s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        t.render_device(u, reg, fr.data_ptr(), w, 0, s)
    torch.cuda.synchronize()
    print(f"reserve={reserve}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms per frame")
    t.close()
    del fr
