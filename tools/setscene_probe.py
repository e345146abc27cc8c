#!/usr/bin/env python3
"""Host time of rt4_context_set_scene: the first scene of a process, further new
scenes (perturbed radii and sun size: new constants to verify), repeats, and a second context.
Usage (GPU box): python tools/setscene_probe.py"""
import ctypes
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    torch.cuda.init()
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    t0 = time.perf_counter()
    tr = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT)
    print(f"context: {(time.perf_counter() - t0) * 1e3:.2f} ms")

    def timed(label, tracer, scene):
        t = time.perf_counter()
        tracer.set_scene(scene)
        print(f"{label}: {(time.perf_counter() - t) * 1e3:.3f} ms")

    base = rt4.Scene.named("sphere")
    timed("set_scene sphere (first scene of the process)", tr, base)
    timed("set_scene sphere (repeat)", tr, base)
    for k in range(1, 4):
        s = rt4.Scene(type(base.desc).from_buffer_copy(base.to_bytes()))
        for i in range(s.desc.n_spheres):
            s.desc.spheres[i].r = ctypes.c_float(s.desc.spheres[i].r * (1.0 + 0.01 * k)).value
        s.desc.sun.angular_size = ctypes.c_float(s.desc.sun.angular_size * (1.0 + 0.003 * k)).value
        timed(f"set_scene sphere with new radii / sun size #{k}", tr, s)
    for name in ("hypercube", "tiger_two_mirrors", "all_primitives"):
        timed(f"set_scene {name} (new)", tr, rt4.Scene.named(name))
    tr2 = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT)
    timed("second context, set_scene sphere (cached constants)", tr2, base)
    tr2.close()
    tr.close()


if __name__ == "__main__":
    main()
